"""GPU: the ChunkFormerModel mirror (chunkformer_amd/model.py) against reference-generated
golden runs -- endless_decode's multi-segment cache carry (chunkformer_model.py:321-459)
and batch_decode's grouping/split (462-552).  Tolerances as tests/test_gpu_parity.py."""
import os

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def small(golden_dir):
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from chunkformer_amd.config import SMALL
    from chunkformer_amd.model import ChunkFormerModel
    from chunkformer_amd.weights import synthetic_state_dict
    g = np.load(os.path.join(golden_dir, "small.npz"))
    sd = synthetic_state_dict(SMALL, int(g["seed"]))
    return g, {dt: ChunkFormerModel(SMALL, sd, dtype=dt) for dt in ("fp32", "bf16", "fp16")}


RELL2 = {"bf16": 2e-2, "fp16": 5e-3}


@pytest.mark.parametrize("dtype", ["fp32", "bf16", "fp16"])
def test_endless_decode_matches_reference(small, dtype):
    from chunkformer_amd.weights import synthetic_features
    g, models = small
    C, L, R, tbd = (int(v) for v in g["endless_clrt"])
    x = synthetic_features([6000], int(g["endless_seed"]))[0]
    ids, eo = models[dtype].endless_decode(x, C, L, R, total_batch_duration=tbd, return_encoder_out=True)
    eo = eo[0].cpu().numpy()
    exp = g["endless_out"]
    assert eo.shape == exp.shape
    ids = ids.reshape(-1).cpu().numpy()
    if dtype == "fp32":
        np.testing.assert_allclose(eo, exp, atol=1e-4, rtol=0)
        assert (ids == g["endless_ids"]).mean() >= 0.999
    else:
        assert np.linalg.norm(eo - exp) / np.linalg.norm(exp) <= RELL2[dtype]
        assert (ids == g["endless_ids"]).mean() >= 0.99


def test_batch_decode_matches_masked_batch(small):
    """batch_decode with a budget that splits case 'a' into several groups returns, per
    utterance, the argmax of the reference's one-shot masked-batch log-probs (batch
    composition does not change an utterance's output)."""
    from chunkformer_amd.model import budget_groups
    from chunkformer_amd.weights import synthetic_features
    g, models = small
    lens = g["a_lens"].tolist()
    C, L, R = (int(v) for v in g["a_clr"])
    xs = synthetic_features(lens, int(g["a_seed"]))
    tbd = 25   # 1249-frame budget -> several groups
    assert len(budget_groups(lens, tbd)) > 1
    hyps = models["fp32"].batch_decode(xs, C, L, R, total_batch_duration=tbd)
    exp = g["a_logp"].argmax(-1)   # [N, C]
    n = g["a_nchunks"].tolist()
    starts = np.cumsum([0] + n)
    for u, h in enumerate(hyps):
        e = exp[starts[u]: starts[u + 1]].reshape(-1)[: int(g["a_outlens"][u])]
        assert h.shape[0] == e.shape[0]
        if e.size == 0:   # a 14-frame utterance subsamples to 0 frames
            continue
        assert (h.cpu().numpy() == e).mean() >= 0.999, f"utt {u}"


def test_encode_returns_lengths(small):
    from chunkformer_amd.weights import synthetic_features
    g, models = small
    lens = g["pc_lens"].tolist()
    xs = synthetic_features(lens, int(g["pc_seed"]))
    xp = torch.zeros(len(lens), max(lens), 80)
    for i, t in enumerate(xs):
        xp[i, : t.shape[0]] = t
    out, ol = models["fp32"].encode(xp, torch.tensor(lens), 16, 32, 32)
    np.testing.assert_allclose(out.cpu().numpy(), g["pc_out"], atol=1e-4, rtol=0)
    assert ol.tolist() == g["pc_mask"].squeeze(1).sum(-1).tolist()


@pytest.mark.parametrize("dtype", ["fp32", "bf16", "fp16"])
def test_endless_graph_replay_equals_eager(small, dtype):
    """configs[3] path: the HIP-graph-replayed middle segments (streaming.py) give exactly the
    eager segment loop's encoder rows and ids (same kernels, same plans, caches carried)."""
    from chunkformer_amd.weights import synthetic_features
    g, models = small
    C, L, R, tbd = (int(v) for v in g["endless_clrt"])
    x = synthetic_features([6000], int(g["endless_seed"]))[0]
    m = models[dtype]
    ids_e, eo_e = m.endless_decode(x, C, L, R, total_batch_duration=tbd, return_encoder_out=True, cuda_graph=False,
                                   pipeline=False)
    ca_e = [c.clone() for c in m.last_endless_caches]
    ids_g, eo_g = m.endless_decode(x, C, L, R, total_batch_duration=tbd, return_encoder_out=True, cuda_graph=True,
                                   pipeline=False)
    assert eo_g.shape == eo_e.shape
    assert torch.equal(eo_g, eo_e)
    assert torch.equal(ids_g, ids_e)
    # segments in flight on several streams, eagerly (EndlessPipeline) and with every segment
    # replayed from one HIP graph (EndlessGraphPipeline, twice: captured, then reused), at depths
    # 2, 3 (default) and 4: same rows, ids and caches
    for graph, depth in ((False, 3), (True, 3), (True, 3), (True, 2), (True, 4)):
        ids_p, eo_p = m.endless_decode(x, C, L, R, total_batch_duration=tbd, return_encoder_out=True, pipeline=True,
                                       cuda_graph=graph, pipeline_depth=depth)
        assert torch.equal(eo_p, eo_e), (graph, depth)
        assert torch.equal(ids_p, ids_e), (graph, depth)
        for a, b in zip(m.last_endless_caches, ca_e):
            assert torch.equal(a, b), (graph, depth)
        if graph:
            runner = next(iter(m._endless_runners.values()))
            assert runner.replayed == len(runner._keep) > 0, depth   # every segment replayed from a graph


def test_endless_tiny_last_segment_matches_reference(small, golden_dir):
    """A last endless segment of 1-22 frames (calc_length <= 0) in every endless mode, fp32, against
    the reference (endless_tail.npz): the rows the reference's Python slice out[:encoder_len] keeps
    (all but one row of the padded chunk at -1, none at 0), ids and final caches."""
    from chunkformer_amd.model import ChunkFormerModel
    from chunkformer_amd.config import SMALL
    from chunkformer_amd.weights import synthetic_features, synthetic_state_dict
    g = np.load(os.path.join(golden_dir, "endless_tail.npz"))
    m = ChunkFormerModel(SMALL, synthetic_state_dict(SMALL, int(g["seed"])), dtype="fp32")
    C, L, R, tbd = (int(v) for v in g["clrt"])
    for n in g["lens"].tolist():
        x = synthetic_features([n], int(g["feat_seed"]))[0]
        for graph, pipe in ((False, False), (True, False), (False, True), (True, True)):
            ids, eo = m.endless_decode(x, C, L, R, total_batch_duration=tbd, return_encoder_out=True, cuda_graph=graph,
                                       pipeline=pipe)
            eo = eo[0].cpu().numpy()
            assert eo.shape == g[f"out_{n}"].shape, (n, graph, pipe)
            np.testing.assert_allclose(eo, g[f"out_{n}"], atol=1e-4, rtol=0, err_msg=str((n, graph, pipe)))
            assert (ids.reshape(-1).cpu().numpy() == g[f"ids_{n}"]).mean() >= 0.99, (n, graph, pipe)
            att, cnn = m.last_endless_caches
            np.testing.assert_allclose(att.cpu().numpy(), g[f"att_{n}"], atol=1e-4, rtol=0)
            np.testing.assert_allclose(cnn.cpu().numpy(), g[f"cnn_{n}"], atol=1e-4, rtol=0)


def test_batch_decode_tiny_utterances_matches_reference(small, golden_dir):
    """batch_decode with utterances of 3-15 frames (tiny_batch.npz): the reference's per-utterance
    rows hyp.flatten()[:x_len] (calc_length -1 keeps all but the last id of the padded chunk, 0 none),
    as ids and as get_output strings (fp32)."""
    from chunkformer_amd.weights import synthetic_features, synthetic_vocab
    g = np.load(os.path.join(golden_dir, "tiny_batch.npz"))
    m = small[1]["fp32"]
    C, L, R = (int(v) for v in g["clr"])
    xs = synthetic_features(g["lens"].tolist(), int(g["feat_seed"]))
    exp = np.split(g["hyps"], np.cumsum(g["hyp_lens"])[:-1])
    mg = np.split(g["margins"], np.cumsum(g["hyp_lens"])[:-1])
    saved = m.char_dict
    try:
        m.char_dict = None
        hyps = m.batch_decode(xs, C, L, R, total_batch_duration=1800)
        assert [h.numel() for h in hyps] == g["hyp_lens"].tolist()
        for h, e, mm in zip(hyps, exp, mg):
            assert (h.cpu().numpy()[mm > 1e-4] == e[mm > 1e-4]).all()
        m.char_dict = synthetic_vocab(m.config.vocab)
        assert m.batch_decode(xs, C, L, R, total_batch_duration=1800) == g["texts"].tolist()
    finally:
        m.char_dict = saved


@pytest.mark.parametrize("dtype", ["bf16", "fp32"])
def test_endless_graph_pipeline_lengths(small, dtype):
    """The graph-replayed pipeline over inputs of several lengths in a row on one model (streaming.py:
    every segment -- the offset-0 first one, the shared middle plan, the ragged last one -- from captured
    graphs keyed by their plans / lengths / kept rows; buffers growing and the old graphs retired):
    each call bit-identical to the one-segment-at-a-time eager loop, a repeated length replaying
    without a new capture, and every segment replayed from a graph."""
    from chunkformer_amd.weights import synthetic_features
    g, models = small
    C, L, R, tbd = (int(v) for v in g["endless_clrt"])
    m = models[dtype]
    # a 4-frame last segment (900: calc_length -1, the reference keeps 15 rows of its padded chunk), three
    # segments, a ragged tail, the fixture length, a longer one, then lengths again
    seen = {}
    for depth in (4, 3):
        for n, seed in ((900, 1), (2100, 2), (4050, 3), (6000, 4), (9000, 5), (4050, 7), (6000, 6)):
            x = synthetic_features([n], seed)[0]
            ids_e, eo_e = m.endless_decode(x, C, L, R, total_batch_duration=tbd, return_encoder_out=True,
                                           cuda_graph=False, pipeline=False)
            ca_e = [c.clone() for c in m.last_endless_caches]
            ids_p, eo_p = m.endless_decode(x, C, L, R, total_batch_duration=tbd, return_encoder_out=True,
                                           pipeline=True, cuda_graph=True, pipeline_depth=depth)
            assert torch.equal(eo_p, eo_e), (n, depth)
            assert torch.equal(ids_p, ids_e), (n, depth)
            for a_, b_ in zip(m.last_endless_caches, ca_e):
                assert torch.equal(a_, b_), (n, depth)
            runner = next(iter(m._endless_runners.values()))
            assert runner.replayed == len(runner._keep) > 0, (n, depth)
            if (depth, n) in seen:   # the same length again: its graphs are reused, none captured
                assert runner.captures == seen[(depth, n)], (n, depth)
            seen[(depth, n)] = runner.captures
            assert len(runner.graphs) <= runner.max_graphs


def test_endless_graphs_bounded_over_many_lengths(small):
    """A long-lived process decoding many distinct input lengths (a service) holds a bounded number of
    captured graphs and device plans: the least recently replayed graph is destroyed once the runner
    holds max_graphs, a replaced runner destroys its own, and every call stays bit-identical to the
    eager loop.  Replacing runners in between (pipeline depth / mode changes) destroys their graphs too."""
    from chunkformer_amd.weights import synthetic_features
    g, models = small
    C, L, R, tbd = (int(v) for v in g["endless_clrt"])
    m = models["fp32"]
    lens = [2100 + 97 * i for i in range(14)]
    xs = [synthetic_features([n], 300 + i)[0] for i, n in enumerate(lens)]
    for depth in (4, 2):
        res = []
        for n, x in zip(lens, xs):   # one runner throughout: its graphs are evicted, not the runner replaced
            res.append(m.endless_decode(x, C, L, R, total_batch_duration=tbd, return_encoder_out=True,
                                        cuda_graph=True, pipeline=True, pipeline_depth=depth))
            runner = next(iter(m._endless_runners.values()))
            assert runner.replayed == len(runner._keep) > 0
            assert len(runner.graphs) <= runner.max_graphs, (n, depth)
            live = {p for key in runner.graphs for p, *_ in key[1]}
            assert {e[2] for e in runner.plans.values()} <= live | {s_["pid"] for s_ in runner._keep}
        assert runner.captures >= len(lens) > runner.max_graphs   # graphs were destroyed along the way
        for n, x, (ids_p, eo_p) in zip(lens, xs, res):   # (replaces the graph runner: its graphs destroyed)
            ids_e, eo_e = m.endless_decode(x, C, L, R, total_batch_duration=tbd, return_encoder_out=True,
                                           cuda_graph=False, pipeline=False)
            assert torch.equal(eo_p, eo_e) and torch.equal(ids_p, ids_e), (n, depth)


@pytest.mark.parametrize("dtype", ["fp32", "bf16", "fp16"])
def test_endless_decode_larger_segments_match_reference(small, golden_dir, dtype):
    """The same input with total_batch_duration 80 (2 segments; the bench runs configs[3] with
    larger segments than the reference default) against the reference run at that tbd
    (endless_tbd80.npz).  The reference's own output moves slightly with the segmentation
    (tests/test_oracle_golden.py::test_reference_endless_depends_on_segmentation)."""
    from chunkformer_amd.weights import synthetic_features
    _, models = small
    g = np.load(os.path.join(golden_dir, "endless_tbd80.npz"))
    C, L, R, tbd = (int(v) for v in g["clrt"])
    x = synthetic_features([6000], int(g["feat_seed"]))[0]
    ids, eo = models[dtype].endless_decode(x, C, L, R, total_batch_duration=tbd, return_encoder_out=True)
    eo, exp = eo[0].cpu().numpy(), g["out"]
    assert eo.shape == exp.shape
    ids = ids.reshape(-1).cpu().numpy()
    if dtype == "fp32":
        np.testing.assert_allclose(eo, exp, atol=1e-4, rtol=0)
        assert (ids == g["ids"]).mean() >= 0.999
        att, cnn = models[dtype].last_endless_caches
        np.testing.assert_allclose(att.cpu().numpy(), g["att"], atol=1e-4, rtol=0)
        np.testing.assert_allclose(cnn.cpu().numpy(), g["cnn"], atol=1e-4, rtol=0)
    else:
        assert np.linalg.norm(eo - exp) / np.linalg.norm(exp) <= RELL2[dtype]
        assert (ids == g["ids"]).mean() >= 0.99


@pytest.mark.parametrize("dtype", ["fp32", "bf16", "fp16"])
def test_endless_trim_equals_full(small, dtype):
    """endless_decode's truncated segments computing only the rows their kept rows depend on (native
    "trim_right", model.endless_trim) give exactly the rows, ids and final caches of the full
    computation, in the one-segment-at-a-time loop and in the graph-replayed pipeline."""
    from chunkformer_amd.weights import synthetic_features
    g, models = small
    x = synthetic_features([6000], int(g["endless_seed"]))[0]
    m = models[dtype]
    # the fixture geometry, R not a multiple of C (24 / 16, 20 / 8), and short segments (tbd 4 / 3: 5-7
    # chunks, so the per-layer reach kept + (nb - 1 - l)(ceil(7/C) + ceil(R/C)) is clamped by n_ch)
    geoms = [tuple(int(v) for v in g["endless_clrt"]), (16, 32, 24, 4), (8, 16, 20, 3)]
    try:
        for C, L, R, tbd in geoms:
            for graph, pipe in ((False, False), (True, False), (True, True)):
                res = {}
                for trim in (False, True):
                    m.endless_trim = trim
                    ids, eo = m.endless_decode(x, C, L, R, total_batch_duration=tbd, return_encoder_out=True,
                                               cuda_graph=graph, pipeline=pipe)
                    res[trim] = (ids, eo, [c.clone() for c in m.last_endless_caches])
                (i0, e0, c0), (i1, e1, c1) = res[False], res[True]
                assert torch.equal(e0, e1), (C, L, R, tbd, graph, pipe)
                assert torch.equal(i0, i1), (C, L, R, tbd, graph, pipe)
                for a, b in zip(c0, c1):
                    assert torch.equal(a, b), (C, L, R, tbd, graph, pipe)
    finally:
        m.endless_trim = True


@pytest.mark.parametrize("seed", range(6))
def test_random_endless_matches_oracle(small, seed):
    """endless_decode on seeded random lengths, total_batch_duration and chunk / context sizes, in the
    default mode (graph-replayed pipeline from 3 segments up) and the eager loop, fp32 against the
    oracle's segment loop (tests/test_oracle_golden.py:oracle_endless): rows at 1e-4, final caches."""
    from test_oracle_golden import oracle_endless
    from chunkformer_amd.config import SMALL
    from chunkformer_amd.weights import synthetic_features, synthetic_state_dict
    rng = np.random.default_rng(4000 + seed)
    n = int(rng.integers(200, 9000))
    tbd = int(rng.choice([6, 10, 20, 35]))
    C = int(rng.choice([8, 16, 32]))
    L, R = int(rng.choice([8, 16, 32])), int(rng.choice([0, 8, 16, 32]))
    x = synthetic_features([n], 1100 + seed)[0]
    m = small[1]["fp32"]
    exp, ac, cc, nseg = oracle_endless(synthetic_state_dict(SMALL, 1), SMALL, x, C, L, R, tbd)
    for kw in ({}, dict(cuda_graph=False, pipeline=False), dict(cuda_graph=True, pipeline=True)):
        _, eo = m.endless_decode(x, C, L, R, total_batch_duration=tbd, return_encoder_out=True, **kw)
        assert eo.shape[1] == exp.shape[0], (n, tbd, C, L, R, nseg, kw)
        np.testing.assert_allclose(eo[0].cpu().numpy(), exp.numpy(), atol=1e-4, rtol=0,
                                   err_msg=str((n, tbd, C, L, R, nseg, kw)))
        att, cnn = m.last_endless_caches
        np.testing.assert_allclose(att.cpu().numpy(), ac.numpy(), atol=1e-4, rtol=0)
        np.testing.assert_allclose(cnn.cpu().numpy(), cc.numpy(), atol=1e-4, rtol=0)


@pytest.mark.parametrize("dtype", ["fp32", "bf16", "fp16"])
def test_endless_fe_reuse_equals_recompute(small, dtype):
    """The graph pipeline carrying each segment's last complete front-end windows into the next
    segment (native fe_carry / fe_reuse / fe_save_from, model.endless_fe_reuse) gives exactly the rows,
    ids and caches of recomputing them, over several input lengths."""
    from chunkformer_amd.weights import synthetic_features
    g, models = small
    C, L, R, tbd = (int(v) for v in g["endless_clrt"])
    m = models[dtype]
    try:
        for n in (6000, 2100, 9000):
            x = synthetic_features([n], 40 + n)[0]
            res = []
            for reuse in (False, True):
                m.endless_fe_reuse = reuse
                ids, eo = m.endless_decode(x, C, L, R, total_batch_duration=tbd, return_encoder_out=True,
                                           cuda_graph=True, pipeline=True)
                res.append((ids, eo, [c.clone() for c in m.last_endless_caches]))
                if reuse:
                    runner = next(iter(m._endless_runners.values()))
                    assert sum(s_["reuse"] for s_ in runner._keep) > 0, n   # windows were carried
            assert torch.equal(res[0][1], res[1][1]) and torch.equal(res[0][0], res[1][0]), n
            for a, b in zip(res[0][2], res[1][2]):
                assert torch.equal(a, b), n
    finally:
        m.endless_fe_reuse = True
