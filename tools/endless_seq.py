"""Replay tests/test_gpu_model.py's test sequence without pytest (the fixture built by hand), to bisect a host
crash in graph replay.   python tools/endless_seq.py [steps]   steps: comma list of m32,m16,mb,g32,gb,g16"""
import faulthandler
import os
import sys

import numpy as np
import torch

faulthandler.enable()
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import test_gpu_model as T  # noqa: E402
from chunkformer_amd.config import SMALL  # noqa: E402
from chunkformer_amd.model import ChunkFormerModel  # noqa: E402
from chunkformer_amd.weights import synthetic_state_dict  # noqa: E402


def main():
    steps = (sys.argv[1] if len(sys.argv) > 1 else "m32,mb,m16,g32,gb,g16").split(",")
    g = np.load(os.path.join(ROOT, "tests", "golden", "small.npz"))
    sd = synthetic_state_dict(SMALL, int(g["seed"]))
    third = os.environ.get("SEQ_THIRD", "fp16")   # the dtype of the model the "16" steps use
    small = (g, {"fp32": ChunkFormerModel(SMALL, sd, dtype="fp32"), "bf16": ChunkFormerModel(SMALL, sd, dtype="bf16"),
                 "fp16": ChunkFormerModel(SMALL, sd, dtype=third)})
    dts = {"32": "fp32", "b": "bf16", "16": "fp16"}
    print("steps", steps, flush=True)
    for s in steps:
        dt = dts[s[1:]]
        if s[0] == "m":
            T.test_endless_decode_matches_reference(small, dt)
        elif s[0] == "g":
            T.test_endless_graph_replay_equals_eager(small, dt)
        else:   # "v": the graph-replay test's calls one by one, with progress
            from chunkformer_amd.weights import synthetic_features
            m = small[1][dt]
            C, L, R, tbd = (int(v) for v in g["endless_clrt"])
            x = synthetic_features([6000], int(g["endless_seed"]))[0]
            for graph, pipe, depth in ((False, False, 3), (True, False, 3), (False, True, 3), (True, True, 3),
                                       (True, True, 3), (True, True, 2), (True, True, 4)):
                print("call", graph, pipe, depth, "runners", list(m._endless_runners), flush=True)
                m.endless_decode(x, C, L, R, total_batch_duration=tbd, return_encoder_out=True, cuda_graph=graph,
                                 pipeline=pipe, pipeline_depth=depth)
                torch.cuda.synchronize()
        torch.cuda.synchronize()
        print("ok", s, flush=True)


if __name__ == "__main__":
    main()
