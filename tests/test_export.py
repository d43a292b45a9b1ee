"""NPZ export/import in the reference's format (exporter.py:78-105) and get_average_colors
(gstex.py:714-726).  CPU only."""
import numpy as np
import torch

from gstex_amd.export import NPZ_KEYS, average_colors, export_npz, load_npz, trainer_from_npz
from gstex_amd.model import GStexTrainer
from gstex_amd.scene import make_scene


def test_npz_round_trip_is_exact(tmp_path):
    sc = make_scene(500, 8000, seed=3)
    tr = GStexTrainer(sc, "cpu")
    with torch.no_grad():
        tr.texture_dc.add_(0.123)  # a non-trivial DC store
    path = tmp_path / "splat.npz"
    export_npz(tr, path)
    with np.load(path, allow_pickle=False) as z:
        assert sorted(z.files) == sorted(NPZ_KEYS)
        assert z["texture_dims"].dtype == np.int32 and z["texture_dims"].shape == (500, 3)
    tr2 = trainer_from_npz(path, "cpu")
    for a, b in [(tr.means, tr2.means), (tr.scales, tr2.scales), (tr.quats, tr2.quats),
                 (tr.opacities, tr2.opacities), (tr.features_rest, tr2.features_rest),
                 (tr.texture_dc, tr2.texture_dc), (tr.texture_dims, tr2.texture_dims), (tr.mappings, tr2.mappings)]:
        assert torch.equal(a.detach(), b.detach())
    assert float(tr2.features_dc.detach().abs().sum()) == 0.0
    assert set(load_npz(path)) == set(NPZ_KEYS)


def test_average_colors_matches_loop():
    g = torch.Generator().manual_seed(1)
    dims = torch.tensor([[2, 3, 0], [1, 1, 6], [4, 2, 7]], dtype=torch.int32)
    tex = torch.randn(15, 3, generator=g)
    avg = average_colors(tex, dims)
    for i, (h, w, off) in enumerate(dims.tolist()):
        ref = (0.28209479177387814 * tex[off:off + h * w] + 0.5).mean(0)
        assert torch.allclose(avg[i], ref, atol=1e-6)
    avg0 = average_colors(tex, dims, sh_degree=0)
    assert torch.allclose(avg0[1], torch.sigmoid(tex[6]), atol=1e-6)
