"""Probe: one masked-batch call of the small / large model under the library CFM_LIB points at, output saved
to gpurun_out/lib_ab_<tag>.pt (compare two runs with --compare).
    CFM_LIB=... python tools/lib_ab_probe.py TAG      |      python tools/lib_ab_probe.py --compare TAG1 TAG2"""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    out_dir = os.path.join(ROOT, "gpurun_out")
    if sys.argv[1] == "--compare":
        a = torch.load(os.path.join(out_dir, f"lib_ab_{sys.argv[2]}.pt"), weights_only=True)
        b = torch.load(os.path.join(out_dir, f"lib_ab_{sys.argv[3]}.pt"), weights_only=True)
        for k in a:
            d = (a[k] - b[k]).abs()
            print(k, "equal" if torch.equal(a[k], b[k]) else f"max {float(d.max()):.3e} differ {int((d > 0).sum())}")
        return
    from chunkformer_amd.config import SMALL
    from chunkformer_amd.encoder import ChunkFormerEncoder
    from chunkformer_amd.weights import synthetic_features, synthetic_state_dict
    g = np.load(os.path.join(ROOT, "tests", "golden", "small.npz"))
    sd = synthetic_state_dict(SMALL, int(g["seed"]))
    res = {}
    for dt in ("bf16", "fp16"):
        enc = ChunkFormerEncoder(SMALL, sd, dtype=dt)
        for case in ("a", "d"):
            lens = g[f"{case}_lens"].tolist()
            C, L, R = (int(v) for v in g[f"{case}_clr"])
            xs = synthetic_features(lens, int(g[f"{case}_seed"]))
            out = enc.forward_parallel_chunk(xs, torch.tensor(lens, dtype=torch.int32), C, L, R)[0]
            res[f"{dt}_{case}"] = out.float().cpu()
    print(SMALL)
    torch.save(res, os.path.join(out_dir, f"lib_ab_{sys.argv[1]}.pt"))


if __name__ == "__main__":
    main()
