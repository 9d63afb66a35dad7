"""In-process A/B timing of model options on the bench workload (one encoder layer or more):
interleaved rounds, per-class event times from libcfm's profiler (cdna guide §5.4 rule 24).

    python tools/ab_bench.py --layers 1 --rounds 3 --variant attn_reuse=0 --variant attn_reuse=1
"""
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
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--minutes", type=float, default=240)
    ap.add_argument("--variant", action="append", default=[])
    ap.add_argument("--heads", type=int, default=8)
    a = ap.parse_args()
    lens = workload_lengths(int(a.minutes * 6000), 0)
    g = torch.Generator(device="cuda").manual_seed(1)
    xs = [torch.randn(t, 80, generator=g, device="cuda") for t in lens]
    from chunkformer_amd.config import LARGE_4H
    cfg = LARGE if a.heads == 8 else LARGE_4H
    enc = ChunkFormerEncoder(cfg, synthetic_state_dict(cfg, 0), dtype="bf16")
    enc.set_option("max_layers", a.layers)
    xl = torch.tensor(lens, dtype=torch.int32)
    variants = [dict(kv.split("=") for kv in v.split(",")) for v in a.variant] or [{}]
    res = [dict() for _ in variants]
    for r in range(a.rounds + 1):
        for vi, v in enumerate(variants):
            for k, val in v.items():
                enc.set_option(k, int(val))
            enc.forward_parallel_chunk(xs, xl, C, L, R)
            torch.cuda.synchronize()
            enc.set_option("profile_reset", 1)
            enc.set_option("profile", (1 << len(_lib.PROFILE_CLASSES)) - 1)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            enc.forward_parallel_chunk(xs, xl, C, L, R)
            e1.record()
            torch.cuda.synchronize()
            enc.set_option("profile", 0)
            if r == 0:
                continue   # warm-up round
            res[vi].setdefault("total", []).append(e0.elapsed_time(e1))
            for k, (ms, n) in _lib.profile_read(enc._h).items():
                if n:
                    res[vi].setdefault(k, []).append(ms)
    for vi, v in enumerate(variants):
        print("variant", v)
        for k, ts in res[vi].items():
            print(f"  {k:20s} median {sorted(ts)[len(ts) // 2]:8.3f} ms  min {min(ts):8.3f}")


if __name__ == "__main__":
    main()
