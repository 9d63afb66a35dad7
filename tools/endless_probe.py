"""Probe: endless_decode modes against the eager one-segment loop for one input length (bit-exact
comparison, first differing row).   python tools/endless_probe.py [frames ...]"""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from chunkformer_amd.config import SMALL  # noqa: E402
from chunkformer_amd.model import ChunkFormerModel  # noqa: E402
from chunkformer_amd.weights import synthetic_features, synthetic_state_dict  # noqa: E402


def first_diff(a, b):
    if a.shape != b.shape:
        return f"shape {tuple(a.shape)} vs {tuple(b.shape)}"
    d = (a != b).reshape(a.shape[0] * a.shape[1], -1).any(-1).nonzero()
    return "equal" if d.numel() == 0 else f"rows {d[0].item()}..{d[-1].item()} differ of {a.shape[1]}"


def main():
    g = np.load(os.path.join(ROOT, "tests", "golden", "small.npz"))
    C, L, R, tbd = (int(v) for v in g["endless_clrt"])
    sd = synthetic_state_dict(SMALL, int(g["seed"]))
    for dt in ("bf16", "fp32"):
        m = ChunkFormerModel(SMALL, sd, dtype=dt)
        for n in [int(a) for a in sys.argv[1:]] or [900, 2100, 4050]:
            x = synthetic_features([n], 1)[0]
            _, ref = m.endless_decode(x, C, L, R, total_batch_duration=tbd, return_encoder_out=True,
                                      cuda_graph=False, pipeline=False)
            for name, kw in (("seq+graph", dict(cuda_graph=True, pipeline=False)),
                             ("pipe eager d3", dict(cuda_graph=False, pipeline=True, pipeline_depth=3)),
                             ("pipe graph d4", dict(cuda_graph=True, pipeline=True, pipeline_depth=4)),
                             ("pipe graph d4 again", dict(cuda_graph=True, pipeline=True, pipeline_depth=4))):
                m.endless_trim = True
                _, eo = m.endless_decode(x, C, L, R, total_batch_duration=tbd, return_encoder_out=True, **kw)
                torch.cuda.synchronize()
                print(dt, n, name, first_diff(eo, ref), flush=True)
            m.endless_trim = False
            _, eo = m.endless_decode(x, C, L, R, total_batch_duration=tbd, return_encoder_out=True,
                                     cuda_graph=False, pipeline=True, pipeline_depth=3)
            print(dt, n, "pipe eager d3 no-trim", first_diff(eo, ref), flush=True)
            m.endless_trim = True


if __name__ == "__main__":
    main()
