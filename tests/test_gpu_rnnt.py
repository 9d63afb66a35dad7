"""GPU: the RNN-T consumer (chunkformer_model.py:439-448 / 533-543) through the
C-ABI (cfm_rnnt_greedy), against the reference's own optimized_search / batch_greedy_search
outputs (tests/golden/rnnt.npz: transducer/search/greedy_search.py:6-92 run by gen_golden.py on
seeded predictor / joint weights over encoder outputs the reference produced) and against the
CPU oracle (oracle/rnnt_ref.py) on random encoder rows with a small n_steps cap.

Tolerance: decisions are integers and must be identical (the golden's smallest top-2 log-prob
margin over every decision is recorded in the fixture, >= 6e-4, far above f32 summation-order
differences)."""
import os

import numpy as np
import pytest
import torch
import yaml

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def rnnt(golden_dir):
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from chunkformer_amd.transducer import RNNTConfig, RNNTGreedy, synthetic_transducer_state_dict
    g = np.load(os.path.join(golden_dir, "rnnt.npz"))
    c = RNNTConfig(vocab=int(g["vocab"]))
    sd = synthetic_transducer_state_dict(c, int(g["seed"]))
    return g, c, sd, RNNTGreedy(c, sd, "cuda")


def _batch_enc(golden_dir, enc_dim):
    g4 = np.load(os.path.join(golden_dir, "large_4h.npz"))
    starts = np.cumsum([0] + g4["nchunks"].tolist())
    return [torch.from_numpy(g4["out"][starts[u]: starts[u + 1]].reshape(-1, enc_dim)[: int(n)])
            for u, n in enumerate(g4["outlens"])]


def test_batch_matches_reference(rnnt, golden_dir):
    g, c, _, dec = rnnt
    utts = _batch_enc(golden_dir, c.enc_dim)
    lens = torch.tensor([u.shape[0] for u in utts])
    enc = torch.nn.utils.rnn.pad_sequence(utts, batch_first=True).cuda()
    out = dec.optimized_search(enc, lens, int(g["n_steps"]))
    np.testing.assert_array_equal(out.cpu().numpy(), g["batch_out"])
    hyps = dec.batch_greedy_search(enc, lens, int(g["n_steps"]))
    assert [len(h) for h in hyps] == g["batch_hyp_lens"].tolist()
    assert [t for h in hyps for t in h] == g["batch_hyps"].tolist()


@pytest.mark.parametrize("grid", [64, 16, 0])
def test_endless_b1_matches_reference(rnnt, golden_dir, grid):
    """B = 1: the multi-CU search (grid_blocks workgroups, grid barriers) and the one-workgroup kernel."""
    g, c, _, dec = rnnt
    ge = np.load(os.path.join(golden_dir, "large_endless.npz"))
    T = g["endless_out"].shape[1] // int(g["n_steps"])
    enc = torch.from_numpy(ge["out"][:T]).unsqueeze(0).cuda()
    dec.set_option("grid_blocks", grid)
    try:
        assert dec.grid_blocks(1) == grid
        out = dec.optimized_search(enc, torch.tensor([T]), int(g["n_steps"]))
    finally:
        dec.set_option("grid_blocks", 64)
    np.testing.assert_array_equal(out.cpu().numpy(), g["endless_out"])


@pytest.mark.parametrize("grid", [64, 0])
@pytest.mark.parametrize("key,n_steps", [("endless_out", 64), ("endless_out_steps3", 3)])
def test_sparse_emission_matches_reference(golden_dir, key, n_steps, grid):
    """rnnt_sparse.npz: a blank-dominated joint (80% of the frames decide blank first, in runs), B=1
    over the endless encoder rows: the regime of the kernel's 8-frame blank-block skip."""
    from chunkformer_amd.transducer import RNNTConfig, RNNTGreedy, synthetic_transducer_state_dict
    g = np.load(os.path.join(golden_dir, "rnnt_sparse.npz"))
    c = RNNTConfig(vocab=int(g["vocab"]))
    sd = synthetic_transducer_state_dict(c, int(g["seed"]), blank_bias=float(g["blank_bias"]),
                                         enc_scale=float(g["enc_scale"]))
    dec = RNNTGreedy(c, sd, "cuda")
    dec.set_option("grid_blocks", grid)
    assert dec.grid_blocks(1) == grid
    ge = np.load(os.path.join(golden_dir, "large_endless.npz"))
    T = g[key].shape[1] // n_steps
    enc = torch.from_numpy(ge["out"][:T]).unsqueeze(0).cuda()
    out = dec.optimized_search(enc, torch.tensor([T]), n_steps)
    np.testing.assert_array_equal(out.cpu().numpy(), g[key])


@pytest.mark.parametrize("grid", [64, 16, 0])
def test_memory_joint_matches_reference(golden_dir, grid):
    """rnnt_memory.npz: a trained-like joint (with_emission_memory) where 95% of the endless rows'
    non-blank frames emit 1-3 tokens and then stop on blank below the n_steps 64 cap (the
    predictor re-evaluated after every emission, the frame loop left on blank); B = 1 on the
    multi-CU search / one workgroup, and the padded batch of two utterances with its hypotheses."""
    from chunkformer_amd.transducer import RNNTGreedy
    from conftest import rnnt_memory_state_dict
    g = np.load(os.path.join(golden_dir, "rnnt_memory.npz"))
    c, sd = rnnt_memory_state_dict(g)
    dec = RNNTGreedy(c, sd, "cuda")
    n = int(g["n_steps"])
    dec.set_option("grid_blocks", grid)
    assert dec.grid_blocks(1) == grid
    ge = np.load(os.path.join(golden_dir, "large_endless.npz"))
    T = g["endless_out"].shape[1] // n
    out = dec.optimized_search(torch.from_numpy(ge["out"][:T]).unsqueeze(0).cuda(), torch.tensor([T]), n)
    np.testing.assert_array_equal(out.cpu().numpy(), g["endless_out"])
    utts = _batch_enc(golden_dir, c.enc_dim)
    lens = torch.tensor([u.shape[0] for u in utts])
    enc = torch.nn.utils.rnn.pad_sequence(utts, batch_first=True).cuda()
    np.testing.assert_array_equal(dec.optimized_search(enc, lens, n).cpu().numpy(), g["batch_out"])
    hyps = dec.batch_greedy_search(enc, lens, n)
    assert [len(h) for h in hyps] == g["batch_hyp_lens"].tolist()
    assert [t for h in hyps for t in h] == g["batch_hyps"].tolist()


@pytest.mark.parametrize("grid", [64, 0])
@pytest.mark.parametrize("n_steps", [1, 3])
def test_small_cap_and_ragged_vs_oracle(rnnt, n_steps, grid):
    """n_steps 1 / 3 (the cap reached often), ragged packed utterances incl. empty and one frame; B = 4
    runs on the multi-CU search (4 x 64 workgroups) or the one-workgroup kernel."""
    from oracle import rnnt_ref
    _, c, sd, dec = rnnt
    gen = torch.Generator().manual_seed(5)
    lens = [37, 0, 1, 90]
    enc = torch.randn(sum(lens), c.enc_dim, generator=gen)
    starts = np.cumsum([0] + lens[:-1]).tolist()
    dec.set_option("grid_blocks", grid)
    try:
        if grid and torch.cuda.get_device_properties(0).multi_processor_count >= 4 * grid:
            assert dec.grid_blocks(len(lens)) == grid
        dense = dec.greedy_packed(enc.cuda(), starts, lens, n_steps).cpu()
    finally:
        dec.set_option("grid_blocks", 64)
    for s0, n in zip(starts, lens):
        o, _ = rnnt_ref.greedy_one(sd, c.num_layers, c.hidden, enc[s0: s0 + n], n_steps)
        np.testing.assert_array_equal(dense[s0: s0 + n].numpy(), o.numpy())


def test_transducer_checkpoint_batch_and_endless(tmp_path, golden_dir, rnnt):
    """A `model: transducer` directory (the vie rnnt recipe: 4-head d=512 encoder, lstm predictor,
    transducer_joint) without a `cmvn` key but with a global_cmvn file (chunkformer_model.py:153-160
    turns CMVN on from the file alone): batch_decode and endless_decode give the reference's RNN-T
    decisions over the same utterances."""
    from chunkformer_amd.config import LARGE_4H, EncoderConfig
    from chunkformer_amd.model import ChunkFormerModel, class2str
    from chunkformer_amd.weights import synthetic_features, synthetic_state_dict, synthetic_vocab
    from test_gpu_checkpoint import ENCODER_CONF
    import json
    g, c, tsd, _ = rnnt
    g4 = np.load(os.path.join(golden_dir, "large_4h.npz"))
    cfg = EncoderConfig(n_heads=4, vocab=c.vocab)
    sd = synthetic_state_dict(LARGE_4H, int(g4["seed"]))   # the golden encoder
    sd.pop("ctc.ctc_lo.weight"), sd.pop("ctc.ctc_lo.bias")
    # CMVN only through the stats file (the checkpoint carries no global_cmvn buffers)
    mean = sd.pop("encoder.global_cmvn.mean").double()
    istd = sd.pop("encoder.global_cmvn.istd").double()
    cnt = 1000.0
    stats = {"mean_stat": (mean * cnt).tolist(), "var_stat": ((1.0 / istd ** 2 + mean ** 2) * cnt).tolist(),
             "frame_num": cnt}
    gen = torch.Generator().manual_seed(11)
    sd["ctc.ctc_lo.weight"] = torch.rand(c.vocab, 512, generator=gen) - 0.5
    sd["ctc.ctc_lo.bias"] = torch.zeros(c.vocab)
    sd.update(tsd)
    conf = {"encoder": "chunkformer", "encoder_conf": ENCODER_CONF, "input_dim": 80, "output_dim": c.vocab,
            "model": "transducer", "predictor": "rnn", "joint": "transducer_joint",
            "predictor_conf": {"embed_size": c.embed_size, "output_size": c.pred_out, "embed_dropout": 0.1,
                               "hidden_size": c.hidden, "num_layers": c.num_layers, "bias": True, "rnn_type": "lstm",
                               "dropout": 0.1},
            "joint_conf": {"enc_output_size": 512, "pred_output_size": c.pred_out, "join_dim": c.join_dim,
                           "prejoin_linear": True, "postjoin_linear": False, "joint_mode": "add", "activation": "tanh"},
            "ctc_conf": {"ctc_blank_id": 0}}
    with open(tmp_path / "config.yaml", "w") as f:
        yaml.safe_dump(conf, f)
    with open(tmp_path / "global_cmvn", "w") as f:
        json.dump(stats, f)
    torch.save(dict(sd), tmp_path / "pytorch_model.bin")
    cd = synthetic_vocab(c.vocab)
    with open(tmp_path / "vocab.txt", "w", encoding="utf8") as f:
        for i, tok in cd.items():
            f.write(f"{tok} {i}\n")
    m = ChunkFormerModel.from_pretrained(str(tmp_path), dtype="fp32")
    assert m.model_type == "transducer" and m.config.cmvn and m.config.n_heads == 4
    xs = synthetic_features(g4["lens"].tolist(), int(g4["feat_seed"]))
    hyps = np.split(g["batch_hyps"], np.cumsum(g["batch_hyp_lens"])[:-1])
    assert m.batch_decode(xs, 64, 128, 128) == [class2str(h, cd).strip() for h in hyps]
    m.char_dict = None
    assert [list(h) for h in m.batch_decode(xs, 64, 128, 128)] == [h.tolist() for h in hyps]
    # utterances of 5 / 3 / 14 frames in the same batch (calc_length -1 / -1 / 0): the reference's
    # optimized_search takes frames t < encoder_out_lens, so they decode to nothing, and the other
    # utterances' hyps do not change (batch composition)
    tiny = synthetic_features([5, 3, 14], 3)
    mixed = m.batch_decode([tiny[0], xs[0], tiny[1]] + list(xs[1:]) + [tiny[2]], 64, 128, 128)
    assert mixed[0] == [] and mixed[2] == [] and mixed[-1] == []
    assert [list(h) for h in [mixed[1]] + mixed[3:-1]] == [h.tolist() for h in hyps]
    n = int(g["n_steps"])
    tok = m.endless_decode(xs[0], 64, 128, 128, total_batch_duration=1800)
    T0 = int(g["batch_lens"][0])
    assert tuple(tok.shape) == (1, T0, n)
    np.testing.assert_array_equal(tok[0].cpu().numpy(), g["batch_out"][0].reshape(-1, n)[:T0])


def test_transducer_endless_segments(rnnt, golden_dir):
    """endless_decode's 4-segment schedule (tbd 20, caches carried, graph replay) feeding the RNN-T
    search: the decisions of the first frames equal the reference's over its own endless output."""
    from chunkformer_amd.config import LARGE
    from chunkformer_amd.model import ChunkFormerModel
    from chunkformer_amd.weights import synthetic_features, synthetic_state_dict
    g, c, tsd, _ = rnnt
    ge = np.load(os.path.join(golden_dir, "large_endless.npz"))
    sd = synthetic_state_dict(LARGE, int(ge["seed"]))
    sd.update(tsd)
    m = ChunkFormerModel(LARGE, sd, dtype="fp32", model_type="transducer", rnnt_config=c)
    x = synthetic_features([int(ge["T"])], int(ge["feat_seed"]))[0]
    Cc, L, R, tbd = (int(v) for v in ge["clrt"])
    tok, eo = m.endless_decode(x, Cc, L, R, total_batch_duration=tbd, return_encoder_out=True)
    n = int(g["n_steps"])
    T = g["endless_out"].shape[1] // n
    assert tok.shape[1] == ge["out"].shape[0]
    np.testing.assert_allclose(eo[0].cpu().numpy(), ge["out"], atol=1e-4, rtol=0)
    np.testing.assert_array_equal(tok[0, :T].cpu().numpy(), g["endless_out"].reshape(-1, n))


@pytest.mark.parametrize("G,B", [(8, 1), (37, 2), (128, 1), (256, 1), (64, 3)])
def test_grid_search_equals_one_workgroup(G, B):
    """The multi-CU search at odd / large workgroup counts (uneven output slices, slices with no
    vocabulary columns) takes exactly the one-workgroup kernel's decisions on random rows, with a
    vocabulary that is not a multiple of 4 (padded columns) and a 1-layer predictor."""
    from chunkformer_amd.transducer import RNNTConfig, RNNTGreedy, synthetic_transducer_state_dict
    c = RNNTConfig(vocab=1001, hidden=256, num_layers=1, embed_size=128, pred_out=256, join_dim=384)
    sd = synthetic_transducer_state_dict(c, 7, blank_bias=5.0)
    dec = RNNTGreedy(c, sd, "cuda")
    if B * G > torch.cuda.get_device_properties(0).multi_processor_count:
        pytest.skip("needs B * G CUs")
    gen = torch.Generator().manual_seed(11)
    lens = [300, 171, 64][:B]
    enc = torch.randn(sum(lens), c.enc_dim, generator=gen).cuda()
    starts = np.cumsum([0] + lens[:-1]).tolist()
    dec.set_option("grid_blocks", 0)
    ref = dec.greedy_packed(enc, starts, lens, 4).cpu()
    dec.set_option("grid_blocks", G)
    assert dec.grid_blocks(B) == G
    # weight slices cached in LDS where they fit (G >= 37 here) or not; exchange by agent-scope
    # atomics (default) or plain accesses behind cache-wide fences
    for lds, atom in ((1, 1), (0, 1), (1, 0)):
        dec.set_option("grid_lds", lds)
        dec.set_option("grid_atomic", atom)
        out = dec.greedy_packed(enc, starts, lens, 4).cpu()
        assert (ref != 0).any() and (ref == 0).any()
        np.testing.assert_array_equal(out.numpy(), ref.numpy())


def test_grid_slices_wider_than_a_workgroup_use_one_workgroup():
    """with G workgroups per utterance every LSTM unit (ceil(H / G)) and projection column quad of a
    workgroup's slice needs a thread of its own (rg_matvec); a small vocabulary with H = 640 at G = 2 would
    give 320 > 256 units per workgroup.  cfm_rnnt_grid_blocks refuses it (0: the one-workgroup kernel), and
    the decisions are the one-workgroup kernel's."""
    from chunkformer_amd.transducer import RNNTConfig, RNNTGreedy, synthetic_transducer_state_dict
    c = RNNTConfig(vocab=200, hidden=640, num_layers=1, embed_size=128, pred_out=256, join_dim=256)
    dec = RNNTGreedy(c, synthetic_transducer_state_dict(c, 3, blank_bias=4.0), "cuda")
    gen = torch.Generator().manual_seed(5)
    enc = torch.randn(90, c.enc_dim, generator=gen).cuda()
    dec.set_option("grid_blocks", 0)
    ref = dec.greedy_packed(enc, [0], [90], 3).cpu()
    for G in (1, 2):
        dec.set_option("grid_blocks", G)
        assert dec.grid_blocks(1) == 0
        np.testing.assert_array_equal(dec.greedy_packed(enc, [0], [90], 3).cpu().numpy(), ref.numpy())
    dec.set_option("grid_blocks", 3)   # ceil(640 / 3) = 214 units per workgroup: the grid kernel runs
    assert dec.grid_blocks(1) == 3
    np.testing.assert_array_equal(dec.greedy_packed(enc, [0], [90], 3).cpu().numpy(), ref.numpy())


def test_grid_barrier_error_falls_back_to_one_workgroup():
    """A multi-CU search that left early (its error word set: a grid barrier that timed out because other
    kernels held CUs) is rerun on the one-workgroup kernel, not returned and not raised."""
    from chunkformer_amd.transducer import RNNTConfig, RNNTGreedy, synthetic_transducer_state_dict
    c = RNNTConfig(vocab=1001, hidden=256, num_layers=1, embed_size=128, pred_out=256, join_dim=384)
    dec = RNNTGreedy(c, synthetic_transducer_state_dict(c, 7, blank_bias=5.0), "cuda")
    gen = torch.Generator().manual_seed(11)
    enc = torch.randn(300, c.enc_dim, generator=gen).cuda()
    dec.set_option("grid_blocks", 0)
    ref = dec.greedy_packed(enc, [0], [300], 4).cpu()
    dec.set_option("grid_blocks", 32)
    dec.set_option("grid_force_error", 1)
    out = dec.greedy_packed(enc, [0], [300], 4).cpu()
    dec.set_option("grid_force_error", 0)
    assert dec.grid_fallbacks == 1 and dec.grid_blocks(1) == 32
    np.testing.assert_array_equal(out.numpy(), ref.numpy())
