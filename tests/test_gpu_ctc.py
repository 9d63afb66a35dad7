"""GPU parity of the fused CTC tail, all through the C-ABI:

  * cfm_ctc_ids (the argmax head that keeps every logit in registers) against a torch fp32 argmax
    of the same bf16-rounded operands, and against the two-pass log-softmax path of the same
    model, for vocabulary sizes at and around the 64-column tile edges, row counts that are not a
    multiple of the 256-row block, and the largest vocabulary the bias image holds (larger V falls
    back to the log-softmax path through the workspace);
  * the CTC ids of the 12-layer large fixture (reference-generated) through the fused head;
  * cfm_ctc_collapse against the CTC oracle (oracle/ctc_ref.py) and the reference's own
    get_output / get_output_with_timestamps output (tests/golden/text.json).

Tolerance: ids are exact wherever the top-2 logit margin exceeds 1e-4 (the fused head and the
references sum the same bf16 products in a different order); collapse/segmentation is integer
work and bit-exact.
"""
import dataclasses
import json
import os

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def _model(V, seed=0, dtype="bf16"):
    from chunkformer_amd.config import LARGE
    from chunkformer_amd.encoder import ChunkFormerEncoder
    from chunkformer_amd.weights import synthetic_state_dict
    cfg = dataclasses.replace(LARGE, vocab=V, num_blocks=1)
    sd = synthetic_state_dict(cfg, seed)
    return ChunkFormerEncoder(cfg, sd, dtype=dtype), sd


def _torch_logits(enc_rows, sd, dtype="bf16"):
    t = torch.float16 if dtype == "fp16" else torch.bfloat16
    w = sd["ctc.ctc_lo.weight"].to(enc_rows.device).to(t).float()
    b = sd["ctc.ctc_lo.bias"].to(enc_rows.device).float()
    return enc_rows.to(t).float() @ w.t() + b


@pytest.fixture(scope="module")
def gen():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    return torch.Generator(device="cuda").manual_seed(5)


@pytest.mark.parametrize("V,rows,dtype", [(5000, 3001, "bf16"), (5000, 256, "bf16"), (37, 700, "bf16"),
                                          (64, 513, "bf16"), (65, 1000, "bf16"), (128, 255, "bf16"),
                                          (7808, 1200, "bf16"), (5000, 3001, "fp16"), (37, 700, "fp16"),
                                          (65, 1000, "fp16"), (7808, 1200, "fp16")])
def test_fused_ids_match_fp32_argmax(gen, V, rows, dtype):
    """The fused head (bf16, or f16 for the fp16 model) against a torch fp32 argmax of the same
    16-bit-rounded operands."""
    enc, sd = _model(V, seed=V, dtype=dtype)
    assert enc.ctc_ws_bytes(rows, False) == 0   # the fused head: no logit workspace
    x = torch.randn(rows, 512, generator=gen, device="cuda") * 1.5
    _, ids = enc.ctc_log_softmax(x, want_logp=False)
    logits = _torch_logits(x, sd, dtype)
    top2 = logits.topk(2, dim=-1).values
    margin = (top2[:, 0] - top2[:, 1]).cpu()
    ref = logits.argmax(-1).int().cpu()
    got = ids.cpu()
    sure = margin > 1e-4
    assert torch.equal(got[sure], ref[sure]), f"{int((got[sure] != ref[sure]).sum())} rows differ"
    assert (got == ref).float().mean() >= 0.999
    assert int(got.min()) >= 0 and int(got.max()) < V
    # the two-pass path of the same model (GEMM -> [rows, V] f32 -> log_softmax) agrees too
    logp, ids2 = enc.ctc_log_softmax(x, want_logp=True)
    assert torch.equal(got[sure], ids2.cpu()[sure])


def test_fused_ids_ties_take_the_lowest_column(gen):
    """Rows whose logits tie exactly (W rows duplicated, zero bias) resolve to the lowest index,
    like torch.argmax."""
    from chunkformer_amd.config import LARGE
    from chunkformer_amd.encoder import ChunkFormerEncoder
    from chunkformer_amd.weights import synthetic_state_dict
    V = 300
    cfg = dataclasses.replace(LARGE, vocab=V, num_blocks=1)
    sd = synthetic_state_dict(cfg, 3)
    w = sd["ctc.ctc_lo.weight"].clone()
    w[250] = w[17]          # column 250 always ties column 17 (different tiles and lanes)
    w[100] = w[99]          # neighbours inside one tile
    sd["ctc.ctc_lo.weight"] = w
    sd["ctc.ctc_lo.bias"] = torch.zeros(V)
    enc = ChunkFormerEncoder(cfg, sd, dtype="bf16")
    x = torch.randn(2048, 512, generator=gen, device="cuda")
    _, ids = enc.ctc_log_softmax(x, want_logp=False)
    ids = ids.cpu()
    assert not bool((ids == 250).any()) and not bool((ids == 100).any())
    logits = _torch_logits(x, sd)
    ref = logits.argmax(-1).int().cpu()
    top2 = logits.topk(2, dim=-1).values
    sure = ((top2[:, 0] - top2[:, 1]) > 1e-4).cpu() | (ref == 17) | (ref == 99)
    assert torch.equal(ids[sure], ref[sure])


def test_vocab_past_the_bias_image_falls_back(gen):
    V = 7809   # 64 * (123 + 2) > 7936: the log-softmax path through the workspace
    enc, sd = _model(V, seed=11)
    assert enc.ctc_ws_bytes(300, False) > 0
    x = torch.randn(300, 512, generator=gen, device="cuda")
    _, ids = enc.ctc_log_softmax(x, want_logp=False)
    logits = _torch_logits(x, sd)
    top2 = logits.topk(2, dim=-1).values
    sure = ((top2[:, 0] - top2[:, 1]) > 1e-4).cpu()
    assert torch.equal(ids.cpu()[sure], logits.argmax(-1).int().cpu()[sure])


def test_fused_ids_on_the_large_fixture():
    """12-layer chunkformer-large, golden utterances: the fused head's ids equal the reference's
    CTC argmax wherever its top-2 margin exceeds 1e-3 (bf16 encoder: >= 99% overall)."""
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from chunkformer_amd.config import LARGE
    from chunkformer_amd.encoder import ChunkFormerEncoder
    from chunkformer_amd.weights import synthetic_features, synthetic_state_dict
    from conftest import GOLDEN
    g = np.load(os.path.join(GOLDEN, "large.npz"))
    sd = synthetic_state_dict(LARGE, int(g["seed"]))
    enc = ChunkFormerEncoder(LARGE, sd, dtype="bf16")
    lens = g["lens"].tolist()
    xs = synthetic_features(lens, int(g["feat_seed"]))
    out = enc.forward_parallel_chunk(xs, torch.tensor(lens, dtype=torch.int32), 64, 128, 128)[0]
    _, ids = enc.ctc_log_softmax(out, want_logp=False)
    _, ids2 = enc.ctc_log_softmax(out, want_logp=True)
    ids = ids.cpu().numpy()
    assert (ids == g["ids"]).mean() >= 0.99
    # same encoder output, two CTC heads: identical except where the logits nearly tie
    lp = enc.ctc_log_softmax(out, want_logp=True)[0]
    t2 = lp.topk(2, dim=-1).values
    sure = ((t2[..., 0] - t2[..., 1]) > 1e-4).cpu().numpy()
    np.testing.assert_array_equal(ids[sure], ids2.cpu().numpy()[sure])


# ------------------------------------------------------------------------------------ collapse
@pytest.fixture(scope="module")
def small_enc():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from chunkformer_amd.config import SMALL
    from chunkformer_amd.encoder import ChunkFormerEncoder
    from chunkformer_amd.weights import synthetic_state_dict
    return ChunkFormerEncoder(SMALL, synthetic_state_dict(SMALL, 1), dtype="bf16")


def _random_streams(rng, lens, V=50):
    out = []
    for n in lens:
        ids = []
        while len(ids) < n:
            if rng.random() < 0.5:
                ids += [0] * int(rng.integers(1, 20))
            else:
                ids += [int(rng.integers(1, V))] * int(rng.integers(1, 4))
        out.append(ids[:n])
    return out


def _pack(streams, gap=5):
    """Utterances at non-adjacent row ranges of one id tensor (gaps filled with junk ids)."""
    starts, flat = [], []
    for s in streams:
        flat += [7] * gap
        starts.append(len(flat))
        flat += s
    return torch.tensor(flat + [7] * gap, dtype=torch.int32), starts, [len(s) for s in streams]


def test_collapse_matches_oracle(small_enc):
    from oracle.ctc_ref import gen_ctc_peak_time, remove_duplicates_and_blank
    rng = np.random.default_rng(3)
    lens = [0, 1, 2, 3, 17, 511, 512, 513, 1500, 100_003]
    streams = _random_streams(rng, lens) + [[0] * 900, [5] * 777, [0, 3, 3, 0, 3, 0]]
    ids, starts, ls = _pack(streams)
    got = small_enc.ctc_collapse(ids.cuda(), starts, ls)
    for s, (toks, frames) in zip(streams, got):
        assert toks == remove_duplicates_and_blank(s)
        assert frames == gen_ctc_peak_time(s)


@pytest.mark.parametrize("ms", [0, 1, 2, 6, 12, 1 << 30])
def test_segments_match_oracle(small_enc, ms):
    from oracle.ctc_ref import segments_with_timestamps
    rng = np.random.default_rng(ms % 97)
    lens = [0, 1, 5, 64, 700, 3000, 40_000]
    streams = _random_streams(rng, lens) + [[0] * 50, [0, 0, 9, 0, 0, 0, 0, 0, 0, 0, 9, 9, 0], [4] * 30]
    ids, starts, ls = _pack(streams)
    got = small_enc.ctc_collapse(ids.cuda(), starts, ls, max_silence=ms)
    for s, segs in zip(streams, got):
        assert segs == segments_with_timestamps(s, ms), (len(s), ms)


def test_collapse_matches_reference_text_golden(small_enc, golden_dir):
    """Device collapse + host class2str reproduce the reference's get_output and
    get_output_with_timestamps strings (tests/golden/text.json, made by model_utils itself)."""
    from chunkformer_amd.model import class2str, format_segments, max_silence_frames
    from chunkformer_amd.weights import synthetic_vocab
    with open(os.path.join(golden_dir, "text.json"), encoding="utf8") as f:
        g = json.load(f)
    cd = synthetic_vocab(int(g["V"]))
    ids, starts, ls = _pack(g["streams"])
    got = small_enc.ctc_collapse(ids.cuda(), starts, ls)
    assert [class2str(t, cd).strip() for t, _ in got] == g["get_output"]
    for ms, exp in g["timestamps"].items():
        segs = small_enc.ctc_collapse(ids.cuda(), starts, ls, max_silence=max_silence_frames(float(ms)))
        assert [format_segments(s, cd) for s in segs] == exp, ms
