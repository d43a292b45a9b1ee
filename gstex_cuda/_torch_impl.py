"""gstex_cuda._torch_impl — the reference API's pure-torch helpers (imported at
nerfstudio/models/gstex.py:28 and models/jagged_texture.py:8).

These are small device-agnostic torch functions the reference calls directly from model code
(e.g. get_uv_mapping, gstex.py:975-990, runs quat_to_rotmat on the GPU every step), not a
fallback for the HIP rasterizer.
"""
import torch
import torch.nn.functional as F


def normalized_quat_to_rotmat(quat: torch.Tensor) -> torch.Tensor:
    """Unit wxyz quaternion (..., 4) -> rotation matrix (..., 3, 3)."""
    w, x, y, z = torch.unbind(quat, dim=-1)
    mat = torch.stack(
        [
            1 - 2 * (y**2 + z**2),
            2 * (x * y - w * z),
            2 * (x * z + w * y),
            2 * (x * y + w * z),
            1 - 2 * (x**2 + z**2),
            2 * (y * z - w * x),
            2 * (x * z - w * y),
            2 * (y * z + w * x),
            1 - 2 * (x**2 + y**2),
        ],
        dim=-1,
    )
    return mat.reshape(quat.shape[:-1] + (3, 3))


def quat_to_rotmat(quat: torch.Tensor) -> torch.Tensor:
    """wxyz quaternion (normalised first) -> rotation matrix (..., 3, 3)."""
    return normalized_quat_to_rotmat(F.normalize(quat, dim=-1))


def sample_texture(query_dims: torch.Tensor, texture: torch.Tensor, uv: torch.Tensor) -> torch.Tensor:
    """Bilinear lookup of each row's texel block [off, off + h*w) (row-major i along u, j along v)
    at uv in [0,1]^2, corner-aligned (texel (i,j) at (i/h, j/w), matching texture_dims_to_query,
    jagged_texture.py:23-34), clamp-to-edge.  Same sampler as the HIP rasterizer."""
    qd = query_dims.long()
    h, w, off = qd[:, 0], qd[:, 1], qd[:, 2]
    has = (h * w) > 0
    hf, wf = h.to(texture.dtype), w.to(texture.dtype)
    x = torch.minimum(torch.clamp(uv[:, 0] * hf, min=0.0), hf - 1)
    y = torch.minimum(torch.clamp(uv[:, 1] * wf, min=0.0), wf - 1)
    i0 = torch.where(has, x, torch.zeros_like(x)).clamp(min=0).long()
    j0 = torch.where(has, y, torch.zeros_like(y)).clamp(min=0).long()
    i1 = torch.minimum(i0 + 1, (h - 1).clamp(min=0))
    j1 = torch.minimum(j0 + 1, (w - 1).clamp(min=0))
    ax = (x - i0.to(x.dtype))[:, None]
    ay = (y - j0.to(y.dtype))[:, None]
    n_tex = max(texture.shape[0], 1)

    def fetch(ii, jj):
        idx = torch.where(has, off + ii * w + jj, torch.zeros_like(ii)).clamp(0, n_tex - 1)
        return texture[idx]

    if texture.shape[0] == 0:
        return torch.zeros((qd.shape[0], texture.shape[1]), dtype=texture.dtype, device=texture.device)
    top = (1 - ay) * fetch(i0, j0) + ay * fetch(i0, j1)
    bot = (1 - ay) * fetch(i1, j0) + ay * fetch(i1, j1)
    out = (1 - ax) * top + ax * bot
    return torch.where(has[:, None], out, torch.zeros_like(out))
