"""Max |enc - golden| of the fp32 path on tests/golden/large.npz (12 layers) and the CTC-id agreement
outside small top-2 margins: sizes the tolerance of tests/test_gpu_parity.py::test_large_12L."""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from chunkformer_amd.encoder import ChunkFormerEncoder  # noqa: E402
from chunkformer_amd.config import LARGE  # noqa: E402
from chunkformer_amd.weights import synthetic_features, synthetic_state_dict  # noqa: E402

g = np.load(os.path.join(ROOT, "tests", "golden", "large.npz"))
enc = ChunkFormerEncoder(LARGE, synthetic_state_dict(LARGE, int(g["seed"])), dtype="fp32")
lens = g["lens"].tolist()
xs = synthetic_features(lens, int(g["feat_seed"]))
out, *_ = enc.forward_parallel_chunk(xs, torch.tensor(lens, dtype=torch.int32), 64, 128, 128)
o = out.cpu().numpy()
_, ids = enc.ctc_log_softmax(out, want_logp=False)
ids = ids.cpu().numpy()
margin = g["top2"][..., 0] - g["top2"][..., 1]
print("max_abs", float(np.abs(o - g["out"]).max()), "p99.99", float(np.quantile(np.abs(o - g["out"]), 0.9999)))
for th in (1e-4, 1e-3):
    sure = margin > th
    print("ids mismatches with margin >", th, int((ids[sure] != g["ids"][sure]).sum()))
