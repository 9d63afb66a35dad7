"""bf16-path accuracy probe: rel-L2 of the encoder output and CTC argmax agreement against the
reference-generated large (12-layer) golden fixture; run once per A/B setting (env knobs are read
once per process).    python tools/bf16_err.py"""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from chunkformer_amd.config import LARGE  # noqa: E402
from chunkformer_amd.encoder import ChunkFormerEncoder  # noqa: E402
from chunkformer_amd.weights import synthetic_features, synthetic_state_dict  # noqa: E402

g = np.load(os.path.join(ROOT, "tests", "golden", "large.npz"))
enc = ChunkFormerEncoder(LARGE, synthetic_state_dict(LARGE, int(g["seed"])), dtype="bf16")
lens = g["lens"].tolist()
xs = synthetic_features(lens, int(g["feat_seed"]))
out, _, _, _, _, _ = enc.forward_parallel_chunk(xs, torch.tensor(lens, dtype=torch.int32), 64, 128, 128)
_, ids = enc.ctc_log_softmax(out, want_logp=False)
o = out.cpu().double().numpy()
rel = np.linalg.norm(o - g["out"]) / np.linalg.norm(g["out"])
print(f"bf16 rel-L2 {rel:.3e}  argmax agreement {(ids.cpu().numpy() == g['ids']).mean():.4f}")
