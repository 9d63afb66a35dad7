"""Probe: the front-end alone (max_layers 0) with fe_fuse_dw2 on / off, bf16 and fp16 models, on
a short synthetic batch: rows that differ and the largest difference.   python tools/dw2_probe.py"""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from chunkformer_amd.config import LARGE  # noqa: E402
from chunkformer_amd.encoder import ChunkFormerEncoder  # noqa: E402
from chunkformer_amd.weights import synthetic_features, synthetic_state_dict  # noqa: E402


def main():
    sd = synthetic_state_dict(LARGE, 0)
    xs = synthetic_features([3000, 1234, 6000], 5)
    lens = torch.tensor([x.shape[0] for x in xs], dtype=torch.int32)
    for dt in ("bf16", "fp16"):
        enc = ChunkFormerEncoder(LARGE, sd, dtype=dt)
        for layers in (0, 1):
            enc.set_option("max_layers", layers)
            for wst in (1, 2):
                enc.set_option("gemm_wst", wst)
                outs = []
                for fuse in (0, 1):
                    enc.set_option("fe_fuse_dw2", fuse)
                    outs.append(enc.forward_parallel_chunk(xs, lens, 64, 128, 128)[0].reshape(-1, 512))
                torch.cuda.synchronize()
                bad = (outs[0] != outs[1]).any(dim=1)
                print(dt, "layers", layers, "gemm_wst", wst, "rows differ", int(bad.sum()), "of", bad.numel(),
                      "max", float((outs[0] - outs[1]).abs().max()), flush=True)


if __name__ == "__main__":
    main()
