"""Per-kernel-class timing of ONE encoder layer on the bench workload (240-min masked batch),
via libcfm's in-stream event profiler.  Used for kernel iteration and PMC runs.

    python tools/layer_bench.py [--layers 1] [--iters 3] [--opt key=value ...]"""
import argparse
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from bench import C, L, R, workload_lengths  # noqa: E402
from chunkformer_amd import _lib  # noqa: E402
from chunkformer_amd.config import LARGE  # noqa: E402
from chunkformer_amd.encoder import ChunkFormerEncoder  # noqa: E402
from chunkformer_amd.weights import synthetic_state_dict  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--layers", type=int, default=1)
    ap.add_argument("--iters", type=int, default=3)
    ap.add_argument("--minutes", type=float, default=240)
    ap.add_argument("--opt", action="append", default=[])
    a = ap.parse_args()
    lens = workload_lengths(int(a.minutes * 6000), 0)
    g = torch.Generator(device="cuda").manual_seed(1)
    xs = [torch.randn(t, 80, generator=g, device="cuda") for t in lens]
    enc = ChunkFormerEncoder(LARGE, synthetic_state_dict(LARGE, 0), dtype="bf16")
    enc.set_option("max_layers", a.layers)
    for o in a.opt:
        k, v = o.split("=")
        enc.set_option(k, int(v))
    xl = torch.tensor(lens, dtype=torch.int32)
    enc.forward_parallel_chunk(xs, xl, C, L, R)
    torch.cuda.synchronize()
    enc.set_option("profile_reset", 1)
    enc.set_option("profile", (1 << len(_lib.PROFILE_CLASSES)) - 1)
    for _ in range(a.iters):
        enc.forward_parallel_chunk(xs, xl, C, L, R)
    torch.cuda.synchronize()
    enc.set_option("profile", 0)
    for k, (ms, n) in _lib.profile_read(enc._h).items():
        if n:
            print(f"{k:20s} {ms / a.iters:9.3f} ms/iter  ({n // a.iters} launches)")


if __name__ == "__main__":
    main()
