"""Dump this framework's small256 masked-batch output (C=64 L=R=128) at a compute dtype, for
offline study of the bf16 error against tests/golden/small256.npz (CTC head design).

    python tools/dump_small256.py [bf16|fp32]   -> gpurun_out/small256_<dtype>.npy"""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from chunkformer_amd.config import SMALL256  # noqa: E402
from chunkformer_amd.encoder import ChunkFormerEncoder  # noqa: E402
from chunkformer_amd.weights import synthetic_features, synthetic_state_dict  # noqa: E402


def main():
    dtype = sys.argv[1] if len(sys.argv) > 1 else "bf16"
    g = np.load(os.path.join(ROOT, "tests", "golden", "small256.npz"))
    enc = ChunkFormerEncoder(SMALL256, synthetic_state_dict(SMALL256, int(g["seed"])), dtype=dtype)
    lens = g["lens"].tolist()
    xs = synthetic_features(lens, int(g["feat_seed"]))
    out = enc.forward_parallel_chunk(xs, torch.tensor(lens, dtype=torch.int32), 64, 128, 128)[0]
    o = out.float().cpu().numpy()
    os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
    np.save(os.path.join(ROOT, "gpurun_out", f"small256_{dtype}.npy"), o)
    ref = g["out"]
    print(dtype, "rel-L2", float(np.linalg.norm(o - ref) / np.linalg.norm(ref)),
          "centered rel-L2", float(np.linalg.norm(o - ref) / np.linalg.norm(ref - ref.reshape(-1, ref.shape[-1]).mean(0))))


if __name__ == "__main__":
    main()
