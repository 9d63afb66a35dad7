"""Host logic of the ChunkFormerModel mirror (chunkformer_amd/model.py) -- no GPU:
endless_decode segment schedule, batch_decode budget grouping, CTC text helpers."""
import os

import numpy as np
import pytest
import torch

from chunkformer_amd.model import (budget_groups, endless_segments, format_segments, get_output, max_silence_frames,
                                   milliseconds_to_hhmmssms, remove_duplicates_and_blank, load_json_cmvn)


def _reference_schedule(xs_len, C, L, R, tbd, nb, k=15, sub=8):
    """Literal restatement of chunkformer_model.py:355-435's loop control."""
    lorder = k // 2
    mult = (int(tbd // 0.01) // 2) // C // sub
    trunc = C * mult
    rel = (max(R, lorder) + max(C, max(R, lorder)) * (nb - 1)) * sub
    out = []
    for idx, _ in enumerate(range(0, xs_len, trunc * sub)):
        start = max(trunc * sub * idx, 0)
        end = min(trunc * sub * (idx + 1) + 7, xs_len)
        seg = (start, min(end + rel, xs_len))
        last = C * mult * sub * idx + rel >= xs_len
        out.append((seg, not last))
        if last:
            break
    return trunc, out


@pytest.mark.parametrize("xs_len,C,L,R,tbd,nb", [(6000, 16, 32, 32, 20, 2), (5_760_000, 64, 128, 128, 1800, 12),
                                                 (5_760_000, 64, 128, 128, 14400, 12), (100, 64, 128, 128, 1800, 12),
                                                 (101_895, 64, 128, 128, 1800, 12), (1, 8, 4, 4, 10, 1)])
def test_endless_schedule_matches_reference_loop(xs_len, C, L, R, tbd, nb):
    trunc, segs = endless_segments(xs_len, C, L, R, tbd, nb)
    rt, ref = _reference_schedule(xs_len, C, L, R, tbd, nb)
    assert trunc == rt
    assert [((a, b), k) for a, b, k, _ in segs] == ref
    assert not any(s[3] for s in segs[:-1])


def test_endless_schedule_golden_segment_count(golden_dir):
    g = np.load(f"{golden_dir}/small.npz")
    C, L, R, tbd = (int(v) for v in g["endless_clrt"])
    _, segs = endless_segments(6000, C, L, R, tbd, 2)
    assert len(segs) == int(g["endless_nseg"])


def test_endless_schedule_16h_counts():
    # 65 segments at tbd=1800, 9 at tbd=14400
    assert len(endless_segments(5_760_000, 64, 128, 128, 1800, 12)[1]) == 65
    assert len(endless_segments(5_760_000, 64, 128, 128, 14400, 12)[1]) == 9
    with pytest.raises(ValueError):
        endless_segments(1000, 64, 128, 128, 0.5, 12)


def test_budget_groups():
    # budget = int(tbd // 0.01) // 2 frames; the utterance that crosses it closes the group
    assert budget_groups([100, 100, 100], 3) == [[0, 1], [2]]          # budget 149
    assert budget_groups([148, 1, 5], 3) == [[0, 1], [2]]          # int(3 // 0.01) // 2 = 149
    assert budget_groups([149, 1, 5], 3) == [[0], [1, 2]]
    assert budget_groups([10], 1800) == [[0]]
    assert budget_groups([], 1800) == []
    assert budget_groups([90000, 1, 2], 1800) == [[0], [1, 2]]


def test_text_helpers():
    assert remove_duplicates_and_blank([0, 1, 1, 0, 1, 2, 2, 0]) == [1, 1, 2]
    assert remove_duplicates_and_blank([]) == []
    cd = {0: "<blank>", 1: "▁xin", 2: "▁chào"}
    assert get_output([[1, 1, 0, 2]], cd) == ["xin chào"]
    assert milliseconds_to_hhmmssms(3_723_004) == "01:02:03:004"
    toks = [0, 0, 1, 0, 0, 0, 0, 0, 0, 0, 0, 2, 2, 0]
    from oracle.ctc_ref import segments_with_timestamps
    assert max_silence_frames(0.5) == 6 and max_silence_frames(0.24) == 2 and max_silence_frames(-1) == 1 << 30
    res = format_segments(segments_with_timestamps(toks, max_silence_frames(0.5)), cd)
    # max_silence = 0.5 // 0.08 = 6 frames -> first sentence ends at t=8, second runs to the end
    assert [r["decode"] for r in res] == ["xin", "chào"]
    assert res[0]["start"] == "00:00:00:000" and res[0]["end"] == milliseconds_to_hhmmssms(8 * 80)
    assert res[1]["start"] == milliseconds_to_hhmmssms(max(-(-(11 + 8) // 2), 9) * 80)


def test_json_cmvn(tmp_path):
    import json
    p = tmp_path / "global_cmvn"
    p.write_text(json.dumps({"mean_stat": [2.0, 4.0], "var_stat": [8.0, 20.0], "frame_num": 2}))
    mean, istd = load_json_cmvn(str(p))
    assert mean == [1.0, 2.0]
    assert istd == pytest.approx([1 / np.sqrt(3.0), 1 / np.sqrt(6.0)])


def test_text_helpers_match_reference_golden(golden_dir):
    """get_output and the CTC oracle's sentence split (oracle/ctc_ref.py, the checker of the device
    collapse kernel) + format_segments against the reference's own model_utils run on the same id
    streams (tests/golden/text.json, written by gen_golden.py)."""
    import json

    from chunkformer_amd.model import get_output
    from chunkformer_amd.weights import synthetic_vocab
    from oracle.ctc_ref import remove_duplicates_and_blank as ref_rdb, segments_with_timestamps
    with open(os.path.join(golden_dir, "text.json"), encoding="utf8") as f:
        g = json.load(f)
    cd = synthetic_vocab(int(g["V"]))
    assert get_output(g["streams"], cd) == g["get_output"]
    for s in g["streams"]:
        assert ref_rdb(s) == remove_duplicates_and_blank(s)
    for ms, exp in g["timestamps"].items():
        got = [format_segments(segments_with_timestamps(s, float(ms) // 0.08), cd) for s in g["streams"]]
        assert got == exp, ms


def test_cmvn_loaders_agree(tmp_path):
    """JSON and kaldi-text global_cmvn stats give the same (mean, istd) (utils/cmvn.py:23-98)."""
    import json

    from chunkformer_amd.model import load_json_cmvn, load_kaldi_cmvn
    rng = np.random.default_rng(3)
    cnt = 12345.0
    m = rng.normal(size=80) * cnt
    v = (rng.random(80) + 0.5) * cnt + m * m / cnt
    (tmp_path / "j").write_text(json.dumps({"mean_stat": m.tolist(), "var_stat": v.tolist(), "frame_num": cnt}))
    (tmp_path / "k").write_text("[ " + " ".join(repr(float(x)) for x in m) + f" {cnt!r}\n"
                                + " ".join(repr(float(x)) for x in v) + " 0 ]\n")
    a, b = load_json_cmvn(str(tmp_path / "j")), load_kaldi_cmvn(str(tmp_path / "k"))
    np.testing.assert_allclose(a[0], b[0], rtol=1e-12)
    np.testing.assert_allclose(a[1], b[1], rtol=1e-12)


def test_endless_graph_blocks_schedule():
    """EndlessGraphPipeline's schedule (host logic): every segment exactly once, in order, in blocks
    of at most `block`, all full but the last; a block's phase is its first segment's slot phase."""
    from chunkformer_amd.streaming import graph_blocks
    for n in range(0, 40):
        for block in (1, 2, 3, 12, 128):
            for period in (2, 4, 6):
                blocks = graph_blocks(n, block, period)
                assert [k for k0, cnt, _ in blocks for k in range(k0, k0 + cnt)] == list(range(n))
                assert all(1 <= cnt <= block for _, cnt, _ in blocks)
                assert all(cnt == block for _, cnt, _ in blocks[:-1])
                assert all(ph == k0 % period for k0, _, ph in blocks)
