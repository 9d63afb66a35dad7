"""Micro-benchmark of the projection GEMM (cfm_op_gemm) on the encoder's shapes.

    python tools/gemm_bench.py [--iters 20] [--small]
Prints TFLOP/s per (M, N, K, epilogue) from HIP events around the launches."""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from chunkformer_amd import _lib as L  # noqa: E402

M = 2845 * 64
SHAPES = [  # (name, N, K, epi, act)
    ("ffn_w1", 2048, 512, 0, 2),
    ("ffn_w2", 512, 2048, 0, 0),
    ("qkv", 1536, 512, 3, 0),
    ("out/pw2", 512, 512, 0, 0),
    ("pw1_glu", 1024, 512, 4, 0),
    ("fe_pw1", 512, 512, 0, 1),
    ("ffn_w1_noact", 2048, 512, 0, 0),   # A/B: the FFN w1 shape without / with a cheap activation
    ("ffn_w1_relu", 2048, 512, 0, 1),
]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--small", action="store_true")
    ap.add_argument("--diag", type=int, default=0, help="timing diagnostic of the bf16 kernels (cfm_ops.h)")
    ap.add_argument("--only", default="")
    ap.add_argument("--store", type=int, default=0, help="epilogue store policy (EpiArgs::store_mode: 2 = nt)")
    ap.add_argument("--m", type=int, default=0, help="rows (default: the 240-min batch)")
    ap.add_argument("--wst", type=int, default=0, help="K = 512 weight-stationary kernel: 1 on, 2 on at any M, 7 off")
    a = ap.parse_args()
    st = torch.cuda.current_stream().cuda_stream
    for name, N, K, epi, act in SHAPES:
        if a.only and name not in a.only.split(","):
            continue
        if a.diag in (3, 4, 5, 7) and K != 512:   # those diagnostics exist only in the K = 512 kernel
            continue
        Mr = a.m if a.m else (M if name != "fe_pw1" else 2845 * 2451 // 4)
        A = torch.randn(Mr, K, device="cuda").to(torch.bfloat16)
        W = (torch.randn(N, K, device="cuda") / K ** 0.5).to(torch.bfloat16)
        bias = torch.randn(N, device="cuda")
        out = torch.empty(Mr + 200, max(N, 1024), device="cuda", dtype=torch.bfloat16)
        x = torch.zeros(Mr, N, device="cuda")
        q = torch.empty(Mr, 512, device="cuda", dtype=torch.bfloat16)
        kv = torch.empty(Mr + 300, 1024, device="cuda", dtype=torch.bfloat16)

        def run():
            if epi == 3:
                L.check(L.cfm_op_gemm(1, epi, act, A.data_ptr(), K, W.data_ptr(), K, Mr, N, K, bias.data_ptr(), 1.0,
                                      q.data_ptr(), 512, 128, kv.data_ptr(), 512, None, 0, None, int(a.small) | (a.diag << 8) | (a.store << 16) | (a.wst << 18), st))
            elif epi == 2:
                L.check(L.cfm_op_gemm(1, epi, act, A.data_ptr(), K, W.data_ptr(), K, Mr, N, K, bias.data_ptr(), 0.5,
                                      None, 0, 0, None, 0, x.data_ptr(), N, None, int(a.small) | (a.diag << 8) | (a.store << 16) | (a.wst << 18), st))
            else:
                L.check(L.cfm_op_gemm(1, epi, act, A.data_ptr(), K, W.data_ptr(), K, Mr, N, K, bias.data_ptr(), 1.0,
                                      out.data_ptr(), out.shape[1], 0, None, 0, None, 0, None, int(a.small) | (a.diag << 8) | (a.store << 16) | (a.wst << 18), st))
        for _ in range(3):
            run()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(a.iters):
            run()
        e1.record()
        torch.cuda.synchronize()
        ms = e0.elapsed_time(e1) / a.iters
        tf = 2.0 * Mr * N * K / ms / 1e9
        print(f"{name:10s} M={Mr:7d} N={N:5d} K={K:5d}  {ms*1e3:8.1f} us  {tf:7.1f} TFLOP/s", flush=True)


if __name__ == "__main__":
    main()
