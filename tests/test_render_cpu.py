"""CPU: the procedural dataset's host half and the renderer oracle, pinned to the reference.

tests/golden/render_ref.npz (make_render_goldens.py, made by importing the reference): 30 items
over (seed, simple, rot_only, size) combinations incl. all four lattice types.
  * toycrystals_amd.data.ToyCrystalsDataset.params reproduces the reference's atom centres, sigma,
    y_cat and y_cont BIT-EXACTLY (same generator draws, same fp32 ops; data.py:73-129,171-221);
  * oracle/render_np.py reproduces the reference's float images within 2 ulp of 1.0 and its uint8
    images exactly (data.py:132-153,204-206, build_dataset.py:34)."""
import numpy as np
import pytest

from oracle.render_np import render_item


@pytest.fixture(scope="module")
def gold():
    import os
    here = os.path.dirname(os.path.abspath(__file__))
    g = np.load(os.path.join(here, "golden", "render_ref.npz"), allow_pickle=False)
    return {k: g[k] for k in g.files}


def cases(g):
    for k in range(int(g["n_cases"])):
        yield {n: g[f"c{k}/{n}"] for n in ("meta", "pts", "sigma", "x", "u8", "y_cat", "y_cont")}


def test_host_params_bit_exact(gold):
    from toycrystals_amd.data import ToyCrystalsDataset
    n = 0
    for c in cases(gold):
        seed, idx, simple, rot, size = (int(v) for v in c["meta"])
        ds = ToyCrystalsDataset(1000, size, seed, 4, bool(simple), bool(rot), device="cpu")
        pts, sigma, yc, yv = ds.params(idx)
        assert pts.numpy().shape == c["pts"].shape
        assert np.array_equal(pts.numpy(), c["pts"])
        assert sigma == float(c["sigma"]) and yc == int(c["y_cat"])
        assert np.array_equal(yv.numpy(), c["y_cont"])
        n += 1
    assert n == 30
    assert len({int(c["y_cat"]) for c in cases(gold)}) == 4  # every lattice type covered


def test_oracle_render_vs_reference(gold):
    for c in cases(gold):
        size = int(c["meta"][4])
        x, u8 = render_item(c["pts"], size, size, float(c["sigma"]))
        assert float(np.abs(x - c["x"][0]).max()) <= 2.4e-7
        assert np.array_equal(u8, c["u8"][0])


def test_empty_point_set_renders_zeros():
    x, u8 = render_item(np.zeros((0, 2), np.float32), 8, 8, 1.2)
    assert not x.any() and not u8.any()
