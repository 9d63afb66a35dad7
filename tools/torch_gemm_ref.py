"""Reference point only: hipBLASLt (torch.matmul, bf16) on the encoder's GEMM shapes."""
import torch
M = 2845 * 64
for name, N, K in [("ffn_w1", 2048, 512), ("ffn_w2", 512, 2048), ("qkv", 1536, 512), ("out/pw2", 512, 512),
                   ("pw1_glu", 1024, 512), ("fe_pw1", 512, 512)]:
    Mr = M if name != "fe_pw1" else 2845 * 2451 // 4
    a = torch.randn(Mr, K, device="cuda").bfloat16()
    w = torch.randn(N, K, device="cuda").bfloat16() / K ** 0.5
    for _ in range(3):
        c = a @ w.t()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(20):
        c = a @ w.t()
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / 20
    print(f"{name:10s} M={Mr:7d} N={N:5d} K={K:5d}  {ms*1e3:8.1f} us  {2*Mr*N*K/ms/1e9:7.1f} TFLOP/s", flush=True)
