"""RNN-T consumer, CPU side: the oracle (oracle/rnnt_ref.py) against the reference's own
optimized_search output (tests/golden/rnnt.npz, gen_golden.py gen_rnnt), the transducer branch of
get_output_with_timestamps (model.transducer_segments) against the reference's strings
(tests/golden/text.json), and the config / schema host logic.  Greedy search is causal, so the
oracle runs on a prefix of each utterance (the decisions of those frames are the golden's)."""
import json
import os

import numpy as np
import pytest
import torch

from chunkformer_amd.transducer import RNNTConfig, schema, synthetic_transducer_state_dict
from oracle import rnnt_ref

torch.set_num_threads(min(8, os.cpu_count() or 1))
PREFIX = 24


@pytest.fixture(scope="module")
def rnnt(golden_dir):
    g = np.load(os.path.join(golden_dir, "rnnt.npz"))
    c = RNNTConfig(vocab=int(g["vocab"]))
    return g, c, synthetic_transducer_state_dict(c, int(g["seed"]))


def _batch_enc(golden_dir, enc_dim):
    g4 = np.load(os.path.join(golden_dir, "large_4h.npz"))
    starts = np.cumsum([0] + g4["nchunks"].tolist())
    return [torch.from_numpy(g4["out"][starts[u]: starts[u + 1]].reshape(-1, enc_dim)[: int(n)])
            for u, n in enumerate(g4["outlens"])]


def test_oracle_matches_reference_batch_prefix(rnnt, golden_dir):
    g, c, sd = rnnt
    n = int(g["n_steps"])
    exp = g["batch_out"].reshape(len(g["batch_lens"]), -1, n)
    for u, enc in enumerate(_batch_enc(golden_dir, c.enc_dim)):
        o, margin = rnnt_ref.greedy_one(sd, c.num_layers, c.hidden, enc[:PREFIX], n)
        np.testing.assert_array_equal(o.numpy(), exp[u, :PREFIX], err_msg=f"utt {u}")
        assert margin > 1e-4


def test_oracle_matches_reference_endless_prefix(rnnt, golden_dir):
    g, c, sd = rnnt
    n = int(g["n_steps"])
    ge = np.load(os.path.join(golden_dir, "large_endless.npz"))
    o, _ = rnnt_ref.greedy_one(sd, c.num_layers, c.hidden, torch.from_numpy(ge["out"][:PREFIX]), n)
    np.testing.assert_array_equal(o.numpy(), g["endless_out"].reshape(-1, n)[:PREFIX])


def test_oracle_matches_reference_sparse_emission(golden_dir):
    """rnnt_sparse.npz: blank dominates (80% of the frames decide blank first, in runs)."""
    g = np.load(os.path.join(golden_dir, "rnnt_sparse.npz"))
    c = RNNTConfig(vocab=int(g["vocab"]))
    sd = synthetic_transducer_state_dict(c, int(g["seed"]), blank_bias=float(g["blank_bias"]),
                                         enc_scale=float(g["enc_scale"]))
    ge = np.load(os.path.join(golden_dir, "large_endless.npz"))
    n = int(g["n_steps"])
    T = g["endless_out"].shape[1] // n
    enc = torch.from_numpy(ge["out"][:T])
    first = g["endless_out"].reshape(-1, n)[:, 0]
    assert 0.7 <= (first == 0).mean() < 1.0
    for key, steps in (("endless_out", n), ("endless_out_steps3", 3)):
        o, _ = rnnt_ref.greedy_one(sd, c.num_layers, c.hidden, enc[:3 * PREFIX], steps)
        np.testing.assert_array_equal(o.numpy(), g[key].reshape(-1, steps)[:3 * PREFIX], err_msg=key)


def test_oracle_matches_reference_memory_joint(golden_dir):
    """rnnt_memory.npz: a trained-like joint (with_emission_memory) where most non-blank frames emit
    1-3 tokens and then stop on blank below the cap; the oracle on a prefix of the endless rows and
    of the batch's first utterance, and the regime itself asserted on the whole fixture."""
    from conftest import rnnt_memory_state_dict
    g = np.load(os.path.join(golden_dir, "rnnt_memory.npz"))
    c, sd = rnnt_memory_state_dict(g)
    n = int(g["n_steps"])
    d = g["endless_out"].reshape(-1, n)
    cnt = (d != 0).sum(1)
    nb = cnt[cnt > 0]
    assert 0.2 <= (cnt == 0).mean() <= 0.8 and ((nb >= 1) & (nb <= 3)).mean() >= 0.9 and (nb == n).any()
    ge = np.load(os.path.join(golden_dir, "large_endless.npz"))
    o, margin = rnnt_ref.greedy_one(sd, c.num_layers, c.hidden, torch.from_numpy(ge["out"][:4 * PREFIX]), n)
    np.testing.assert_array_equal(o.numpy(), d[:4 * PREFIX])
    assert margin > 1e-4
    utt0 = _batch_enc(golden_dir, c.enc_dim)[0]
    o, _ = rnnt_ref.greedy_one(sd, c.num_layers, c.hidden, utt0[:2 * PREFIX], n)
    np.testing.assert_array_equal(o.numpy(), g["batch_out"].reshape(len(g["batch_lens"]), -1, n)[0, :2 * PREFIX])


def test_golden_exercises_every_branch(rnnt):
    """The fixture covers blank frames, frames with a few tokens ended by a blank, and frames that
    reach the n_steps cap; the batch hypotheses are the non-blank decisions in order."""
    g, _, _ = rnnt
    n = int(g["n_steps"])
    d = np.concatenate([g["batch_out"].reshape(-1, n), g["endless_out"].reshape(-1, n)])
    cnt = (d != 0).sum(1)
    assert (cnt == 0).any() and ((cnt > 0) & (cnt < n)).any() and (cnt == n).any()
    flat = g["batch_out"].reshape(len(g["batch_lens"]), -1)
    hyps = np.split(g["batch_hyps"], np.cumsum(g["batch_hyp_lens"])[:-1])
    for row, h in zip(flat, hyps):
        np.testing.assert_array_equal(row[row != 0], h)


def test_transducer_timestamps_match_reference(golden_dir):
    from chunkformer_amd.model import format_segments, max_silence_frames, transducer_segments
    from chunkformer_amd.weights import synthetic_vocab
    with open(os.path.join(golden_dir, "text.json"), encoding="utf8") as f:
        text = json.load(f)
    cd = synthetic_vocab(int(text["V"]))
    for ms, exp in text["transducer_timestamps"].items():
        got = [format_segments(transducer_segments(np.array(d, np.int64).reshape(len(d), -1),
                                                   max_silence_frames(float(ms))), cd)
               for d in text["transducer_streams"]]
        assert got == exp, ms


def test_config_from_vie_recipe():
    conf = {"predictor": "rnn", "joint": "transducer_joint",
            "predictor_conf": {"embed_size": 256, "output_size": 512, "embed_dropout": 0.1, "hidden_size": 512,
                               "num_layers": 2, "bias": True, "rnn_type": "lstm", "dropout": 0.1},
            "joint_conf": {"enc_output_size": 512, "pred_output_size": 512, "join_dim": 512, "prejoin_linear": True,
                           "postjoin_linear": False, "joint_mode": "add", "activation": "tanh"}}
    c = RNNTConfig.from_conf(conf, 1024, 512)
    assert (c.embed_size, c.hidden, c.num_layers, c.pred_out, c.join_dim, c.vocab) == (256, 512, 2, 512, 512, 1024)
    names = [n for n, _ in schema(c)]
    assert "predictor.rnn.weight_hh_l1" in names and "joint.ffn_out.bias" in names
    bad = dict(conf, predictor_conf=dict(conf["predictor_conf"], rnn_type="gru"))
    with pytest.raises(AssertionError):
        RNNTConfig.from_conf(bad, 1024, 512)
    with pytest.raises(AssertionError):
        RNNTConfig.from_conf(dict(conf, joint_conf=dict(conf["joint_conf"], postjoin_linear=True)), 1024, 512)
