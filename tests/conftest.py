import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)
GOLDEN = os.path.join(ROOT, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (run via gpurun)")


@pytest.fixture(scope="session")
def golden_dir():
    return GOLDEN


def with_fixture_ctc_head(sd, g):
    """Install the peaked CTC head a fixture recorded (tests/golden/gen_golden.py:peaked_ctc_head):
    the seeded ctc_lo rows scaled by `ctc_rest_scale`, the head's active rows and its bias."""
    import torch
    sd = dict(sd)
    w = sd["ctc.ctc_lo.weight"] * float(g["ctc_rest_scale"])
    w[torch.from_numpy(g["ctc_rows"].astype("int64"))] = torch.from_numpy(g["ctc_w_rows"])
    sd["ctc.ctc_lo.weight"] = w.contiguous()
    sd["ctc.ctc_lo.bias"] = torch.from_numpy(g["ctc_bias"]).contiguous()
    return sd


def rnnt_memory_state_dict(g):
    """(RNNTConfig, state dict) of tests/golden/rnnt_memory.npz (gen_golden.py gen_rnnt_memory)."""
    import torch
    from chunkformer_amd.transducer import RNNTConfig, synthetic_transducer_state_dict, with_emission_memory
    c = RNNTConfig(vocab=int(g["vocab"]))
    sd = with_emission_memory(synthetic_transducer_state_dict(c, int(g["seed"])), c,
                              torch.from_numpy(g["frame_dirs"]), torch.from_numpy(g["frame_bias"]),
                              g["tokens"].tolist(), forget=float(g["forget"]), suppress=float(g["suppress"]))
    return c, sd
