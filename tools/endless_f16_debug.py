"""Isolate a host crash in graph replay of the endless pipeline: the test_gpu_model.py sequence (three models,
endless_decode at default settings, then the (graph, depth) combinations) in child processes, with variants.

    python tools/endless_f16_debug.py"""
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

CHILD = r'''
import faulthandler, gc, sys, numpy as np, torch
faulthandler.enable()
sys.path.insert(0, sys.argv[1])
from chunkformer_amd.config import SMALL
from chunkformer_amd.model import ChunkFormerModel
from chunkformer_amd.weights import synthetic_state_dict, synthetic_features
variant = sys.argv[2]
g = np.load(sys.argv[1] + "/tests/golden/small.npz")
sd = synthetic_state_dict(SMALL, int(g["seed"]))
dts = variant.split(",")[0].split("+")
models = {dt: ChunkFormerModel(SMALL, sd, dtype=dt) for dt in dts}
C, L, R, tbd = (int(v) for v in g["endless_clrt"])
x = synthetic_features([6000], int(g["endless_seed"]))[0]
sync = "sync" in variant
for dt in dts:
    models[dt].endless_decode(x, C, L, R, total_batch_duration=tbd, return_encoder_out=True)
    torch.cuda.synchronize()
print("first calls done", flush=True)
if "bd" in variant:   # test_batch_decode_matches_masked_batch
    lens = g["a_lens"].tolist()
    xs = synthetic_features(lens, int(g["a_seed"]))
    models["fp32"].batch_decode(xs, *(int(v) for v in g["a_clr"]), total_batch_duration=25)
    torch.cuda.synchronize()
    print("batch_decode done", flush=True)
if "enc" in variant:   # test_encode_returns_lengths
    lens = g["pc_lens"].tolist()
    xs = synthetic_features(lens, int(g["pc_seed"]))
    xp = torch.zeros(len(lens), max(lens), 80)
    for i, t in enumerate(xs):
        xp[i, : t.shape[0]] = t
    models["fp32"].encode(xp, torch.tensor(lens), 16, 32, 32)
    torch.cuda.synchronize()
    print("encode done", flush=True)
for dt in dts:
    m = models[dt]
    ids_e, eo_e = m.endless_decode(x, C, L, R, total_batch_duration=tbd, return_encoder_out=True, cuda_graph=False,
                                   pipeline=False)
    m.endless_decode(x, C, L, R, total_batch_duration=tbd, return_encoder_out=True, cuda_graph=True, pipeline=False)
    for graph, depth in ((False, 3), (True, 3), (True, 3), (True, 2), (True, 4)):
        ids_p, eo_p = m.endless_decode(x, C, L, R, total_batch_duration=tbd, return_encoder_out=True, pipeline=True,
                                       cuda_graph=graph, pipeline_depth=depth)
        ok = torch.equal(eo_p, eo_e) and torch.equal(ids_p, ids_e)
        if sync:
            torch.cuda.synchronize()
            gc.collect()
        print(dt, graph, depth, ok, flush=True)
print("done", flush=True)
'''


def main():
    for variant in sys.argv[1:] or ["fp32+bf16+fp16,bd,enc", "fp32+bf16+fp16,bd", "fp32+bf16+fp16,enc"]:
        v = variant.replace("fp16b", "fp16")
        r = subprocess.run([sys.executable, "-c", CHILD, ROOT, v], capture_output=True, text=True, timeout=300)
        out = [l for l in (r.stdout + r.stderr).splitlines() if "amdgpu.ids" not in l]
        print(f"[{variant}] rc={r.returncode}", *out[-14:], sep="\n  ", flush=True)


if __name__ == "__main__":
    main()
