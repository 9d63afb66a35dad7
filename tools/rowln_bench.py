"""Micro-benchmark of the row-owning GEMM with the fused residual + LayerNorm epilogue
(cfm_op_gemm_rowln) against the plain bf16 GEMM of the same shape (cfm_op_gemm, y store only).

    python tools/rowln_bench.py [--iters 20] [--m 182080]
variants: 0 = full epilogue, 1 = no epilogue, 2 = epilogue arithmetic without its loads / stores."""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from chunkformer_amd import _lib as L  # noqa: E402


def timeit(fn, iters):
    for _ in range(3):
        fn()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / iters * 1e3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--m", type=int, default=2845 * 64)
    ap.add_argument("--variants", default="0,1")
    a = ap.parse_args()
    M, N = a.m, 512
    st = torch.cuda.current_stream().cuda_stream
    dev = "cuda"
    for name, K, two in (("ffn_mac_w2+LN_mha", 2048, False), ("linear_out+LN_conv", 512, False),
                         ("ffn_w2+LN_fin+LN_ffm", 2048, True)):
        A = (torch.randn(M, K, device=dev) * 0.5).to(torch.bfloat16)
        W = (torch.randn(N, K, device=dev) / K ** 0.5).to(torch.bfloat16)
        bias = torch.randn(N, device=dev) * 0.1
        x = torch.randn(M, N, device=dev)
        y1 = torch.randn(M, N, device=dev).to(torch.bfloat16)
        h = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
        g1, b1 = torch.ones(N, device=dev), torch.zeros(N, device=dev)
        out = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
        ym = torch.ones(M, device=dev, dtype=torch.uint8)
        yb = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
        for tag, var in (("256x256 tiles", 0), ("128x512 tiles", 1 << 21)):
            us = timeit(lambda: L.check(L.cfm_op_gemm(1, 0, 0, A.data_ptr(), K, W.data_ptr(), K, M, N, K, bias.data_ptr(),
                                                      1.0, out.data_ptr(), N, 0, None, 0, None, 0, None, var, st)),
                        a.iters)
            print(f"{name:24s} K={K:5d} plain GEMM {tag} {us:8.1f} us", flush=True)
        for v in (int(t) for t in a.variants.split(",")):
            def run():
                mac = name.startswith("ffn_mac")   # FFN_mac site: y_out + h, x untouched
                L.check(L.cfm_op_gemm_rowln(A.data_ptr(), K, W.data_ptr(), K, M, K, bias.data_ptr(), 0.5, None,
                                            x.data_ptr(), None if mac else y1.data_ptr(), 1.0,
                                            ym.data_ptr() if two else None, out.data_ptr() if mac else None,
                                            None if mac else x.data_ptr(),
                                            g1.data_ptr(), b1.data_ptr(), g1.data_ptr() if two else None,
                                            b1.data_ptr() if two else None, h.data_ptr(), None, None, yb.data_ptr(), 1e-5, v, st))
            us = timeit(run, a.iters)
            print(f"{name:24s} K={K:5d} rowln variant {v}          {us:8.1f} us", flush=True)


if __name__ == "__main__":
    main()
