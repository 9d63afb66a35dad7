"""CPU-side checks of the C-ABI library: it loads, exports every symbol include/cfm.h
declares, and its HOST planner (no GPU involved) reproduces the reference packer
bit-exactly (golden masks from the reference)."""
import os
import re

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture(scope="module")
def lib():
    from chunkformer_amd import build
    build.build()
    from chunkformer_amd import _lib
    return _lib


def test_exports_every_declared_symbol(lib):
    for h, exported in (("cfm.h", lib.EXPORTED), ("cfm_ops.h", lib.EXPORTED_OPS)):
        hdr = open(os.path.join(ROOT, "include", h)).read()
        declared = set(re.findall(r"\b(cfm_[a-z_]+)\s*\(", hdr))
        assert declared, "no declarations parsed"
        for name in sorted(declared):
            assert hasattr(lib.lib, name), f"libcfm.so does not export {name}"
        assert set(exported) == declared


def test_version(lib):
    assert b"gfx950" in lib.cfm_version()


def _plan_to_masks(plan, C, L, R):
    h = plan[:16]
    N = int(h[1])
    meta = plan[16:16 + 8 * N].reshape(N, 8)
    j = np.arange(L + C + R)[None, :]
    att = (j >= meta[:, 2:3]) & (j < meta[:, 3:4])
    j2 = np.arange(C + 14)[None, :]
    pad = (j2 >= meta[:, 4:5]) & (j2 < meta[:, 5:6])
    return att, pad


def test_planner_bit_exact_vs_reference(lib, golden_dir):
    g = np.load(os.path.join(golden_dir, "masks.npz"))
    for i in range(int(g["n_cases"])):
        C, L, R = (int(v) for v in g[f"c{i}_clr"])
        lens, offs = g[f"c{i}_lens"].tolist(), g[f"c{i}_offs"].tolist()
        plan, nch, olens = lib.plan_masked(lens, offs, C, L, R)
        assert nch == g[f"c{i}_nchunks"].tolist(), f"case {i}"
        assert olens == g[f"c{i}_outlens"].tolist(), f"case {i}"
        att, pad = _plan_to_masks(plan.numpy(), C, L, R)
        sa, sp = g[f"c{i}_att_shape"], g[f"c{i}_pad_shape"]
        exp_att = np.unpackbits(g[f"c{i}_att"], axis=-1, count=int(sa[1])).astype(bool)
        exp_pad = np.unpackbits(g[f"c{i}_pad"], axis=-1, count=int(sp[1])).astype(bool)
        np.testing.assert_array_equal(att, exp_att, err_msg=f"case {i}")
        np.testing.assert_array_equal(pad, exp_pad, err_msg=f"case {i}")


def test_planner_rejects_bad_args(lib):
    with pytest.raises(ValueError):
        lib.plan_masked([100], [0], 0, 4, 4)
    with pytest.raises(ValueError):
        lib.plan_masked([], [], 8, 4, 4)
    with pytest.raises(AssertionError):
        lib.plan_padded([30000], 30000, 5000, 0, 0)


def test_plan_padded_geometry(lib):
    from oracle.encoder_ref import calc_length
    plan, tp = lib.plan_padded([300, 123, 17], 300, 16, 32, 32)
    assert tp == calc_length(300)
    p = plan.numpy()
    assert p[0] == 2 and p[1] == 3 and p[4] == 3 * tp
    plan, tp = lib.plan_padded([300, 123, 17], 300, 0, 0, 0)
    assert p[9] == tp


def test_plan_stream_geometry():
    """cfm_plan_stream (host C++, forward_chunk geometry): key window, rel-pos base, conv chunk edges."""
    from chunkformer_amd import _lib
    C, L, R, off = 16, 32, 16, 5
    T = 8 * (C + R - 1) + 15
    plan, tp = _lib.plan_stream(T, C, L, R, off)
    h = plan[:16].tolist()
    assert tp == C + R and h[0] == 3 and h[4] == tp and h[12] == L + tp and h[13] == 7 + tp
    att = plan[16 + 8: 16 + 8 + 8].tolist()          # the one attention block (T' <= 64)
    assert att[:8] == [0, tp, 0, L - off, L + tp, tp - 1, tp, 0]
    conv = plan[16 + 16: 16 + 16 + 16].view(2, 8).tolist()
    assert conv[0][:5] == [0, C, 0, 0, C + 7] and conv[1][:5] == [C, C, C, 0, C + 7]
    import pytest
    with pytest.raises(ValueError):
        _lib.plan_stream(8 * (C + R) + 15 + 8, C, L, R, 0)   # more than C + R frames
    with pytest.raises(ValueError):
        _lib.plan_stream(8 * 3 + 15, C, L, R, 0)             # fewer than R frames


def test_planner_rows_differ_from_origin_lens(lib, golden_dir):
    """x.size(0) != xs_origin_lens (encoder.py:556-596, 673): windows from the rows, bounds and out
    lengths from xs_origin_lens; a bound count that differs from the window count is the
    reference's shape-mismatch RuntimeError."""
    g = np.load(os.path.join(golden_dir, "rows_neq.npz"))
    C, L, R = (int(v) for v in g["clr"])
    plan, nch, olens = lib.plan_masked(g["rows"].tolist(), [0] * len(g["rows"]), C, L, R, mask_lens=g["lens"].tolist())
    assert nch == g["nchunks"].tolist() and olens == g["outlens"].tolist()
    with pytest.raises(RuntimeError):
        lib.plan_masked([700], [0], C, L, R, mask_lens=[300])
