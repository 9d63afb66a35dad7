"""Timing of the RNN-T greedy consumer (cfm_rnnt_greedy) on synthetic encoder rows: B utterances of
T frames each (B = 1: endless_decode's single long utterance; B > 1: batch_decode), seeded
synthetic predictor / joint weights.  Prints frames/s and emissions per frame.

    python tools/rnnt_bench.py --frames 500 --batch 1
"""
import argparse
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from chunkformer_amd.transducer import RNNTConfig, RNNTGreedy, synthetic_transducer_state_dict  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--frames", type=int, default=45000)
    ap.add_argument("--batch", type=int, default=1)
    ap.add_argument("--grid", type=int, nargs="*", default=[64],
                    help="workgroups per utterance of the multi-CU search (0 = one workgroup)")
    ap.add_argument("--blank-bias", type=float, default=3.72)
    ap.add_argument("--grid-lds", type=int, nargs="*", default=[1], help="weight slices cached in LDS (0 / 1)")
    ap.add_argument("--grid-atomic", type=int, nargs="*", default=[1],
                    help="exchange by agent-scope atomics (1) or fences (0)")
    a = ap.parse_args()
    c = RNNTConfig()
    g = RNNTGreedy(c, synthetic_transducer_state_dict(c, 0, blank_bias=a.blank_bias), device="cuda")
    gen = torch.Generator(device="cuda").manual_seed(3)
    B, T = a.batch, a.frames
    enc = torch.randn(B * T, c.enc_dim, generator=gen, device="cuda")
    starts = [b * T for b in range(B)]
    lens = [T] * B
    ref = None
    for G, lds, atom in [(G, l, at) for G in a.grid for l in a.grid_lds for at in a.grid_atomic]:
        g.set_option("grid_blocks", G)
        g.set_option("grid_lds", lds)
        g.set_option("grid_atomic", atom)
        g.greedy_packed(enc[: min(B * T, 2000)], [0], [min(T, 2000)])   # warm-up
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        out = g.greedy_packed(enc, starts, lens)
        torch.cuda.synchronize()
        dt = time.perf_counter() - t0
        same = "" if ref is None else f", identical to grid {a.grid[0]}: {bool(torch.equal(out, ref))}"
        ref = out if ref is None else ref
        emis = int((out != c.blank).sum().item())
        print(f"grid {G} lds {lds} atomic {atom} (used {g.grid_blocks(B)}) B={B} T={T}: {dt * 1e3:.1f} ms, {B * T / dt:.0f} frames/s, "
              f"{emis / (B * T):.3f} emissions per frame, {dt * 1e3 / max(emis / B, 1):.4f} ms per emission per "
              f"utterance{same}", flush=True)


if __name__ == "__main__":
    main()
