"""Host-side data-format helpers vs golden vectors produced by the REFERENCE's own pure-torch
functions (tests/golden/make_golden.py; jagged_texture.py:10-34, gstex.py:68-99,841-888,975-990)."""
import os

import numpy as np
import pytest
import torch

from gstex_amd import charts

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "host_goldens.npz")


@pytest.fixture(scope="module")
def gold():
    return np.load(GOLD, allow_pickle=False)


def test_random_quat_tensor(gold):
    torch.manual_seed(int(gold["rq_seed"][0]))
    q = charts.random_quat_tensor(64)
    assert np.array_equal(q.numpy(), gold["rq_out"])


def test_sh_rgb_conversions(gold):
    rgb = torch.from_numpy(gold["rgb_in"])
    assert np.array_equal(charts.RGB2SH(rgb).numpy(), gold["rgb2sh_out"])
    assert np.array_equal(charts.SH2RGB(rgb).numpy(), gold["sh2rgb_out"])


@pytest.mark.parametrize("tag", ["a", "b", "c"])
def test_build_charts_matches_reference(gold, tag):
    log_scales = torch.from_numpy(gold[f"bc_{tag}_log_scales"])
    pix = float(gold[f"bc_{tag}_pixel_num"][0])
    dims, mappings, ps = charts.build_charts(log_scales, pix)
    assert np.array_equal(dims.numpy(), gold[f"bc_{tag}_dims"])
    assert np.array_equal(mappings.numpy(), gold[f"bc_{tag}_mappings"])
    assert np.float32(ps) == gold[f"bc_{tag}_pixel_scale"][0]
    total = int((dims[:, 0] * dims[:, 1]).sum())
    assert abs(total - pix) <= 1e-3 * pix  # the bisection's 0.1 % budget (gstex.py:861)


def test_texture_dims_queries_match_reference(gold):
    dims = torch.from_numpy(gold["tq_dims"])
    ids, iuv = charts.texture_dims_to_int_coords(dims)
    assert np.array_equal(ids.numpy(), gold["tq_int_ids"])
    assert np.array_equal(iuv.numpy(), gold["tq_int_uv"])
    qids, quv = charts.texture_dims_to_query(dims)
    assert np.array_equal(qids.numpy(), gold["tq_ids"])
    assert np.array_equal(quv.numpy(), gold["tq_uv"])


def test_uv_mapping_matches_reference(gold):
    quats = torch.from_numpy(gold["uvm_quats"])
    mappings = torch.from_numpy(gold["uvm_mappings"])
    uv0, umap, vmap = charts.get_uv_mapping(quats, mappings)
    assert np.array_equal(uv0.numpy(), gold["uvm_uv0"])
    # reference run used rotations.quaternion_to_matrix (2/|q|^2 form); gstex_cuda's quat_to_rotmat
    # normalises first -> equal up to fp32 rounding
    np.testing.assert_allclose(umap.numpy(), gold["uvm_umap"], rtol=0, atol=2e-6)
    np.testing.assert_allclose(vmap.numpy(), gold["uvm_vmap"], rtol=0, atol=2e-6)


def test_build_charts_zero_budget_raises():
    with pytest.raises(ZeroDivisionError):
        charts.build_charts(torch.zeros(4, 3), 0)
