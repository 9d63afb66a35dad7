"""Which output rows / columns a GEMM variant leaves unwritten (NaN-prefilled) or wrong."""
import os, sys
import torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from chunkformer_amd import _lib as L  # noqa: E402

for (M, N, K, act) in [(70001, 512, 512, 0), (33000, 2048, 512, 2)]:
    g = torch.Generator(device="cuda").manual_seed(1)
    A = (torch.randn(M, K, device="cuda", generator=g) * 0.5).to(torch.bfloat16)
    W = (torch.randn(N, K, device="cuda", generator=g) / K ** 0.5).to(torch.bfloat16)
    bias = torch.randn(N, device="cuda", generator=g)
    out = torch.full((M + 3, N), float("nan"), device="cuda", dtype=torch.bfloat16)
    st = torch.cuda.current_stream().cuda_stream
    L.check(L.cfm_op_gemm(L.DTYPE_BF16, 0, act, A.data_ptr(), K, W.data_ptr(), K, M, N, K, bias.data_ptr(), 1.0,
                          out.data_ptr(), N, 3, None, 0, None, 0, None, 0, st))
    torch.cuda.synchronize()
    r = A.float() @ W.float().t() + bias
    if act == 2:
        r = torch.nn.functional.silu(r)
    o = out[3:].float()
    nan = torch.isnan(o)
    bad = (o - r).abs() > 0.05 * r.abs().max()
    print(f"M={M} N={N} act={act}: nan={int(nan.sum())} bad={int(bad.sum())} pre-rows-nan={bool(torch.isnan(out[:3].float()).all())}")
    for name, m in (("nan", nan), ("bad", bad & ~nan)):
        if m.any():
            rows = m.any(1).nonzero().flatten()
            cols = m.any(0).nonzero().flatten()
            tiles = torch.unique(rows // 64)
            print(f"  {name}: rows {rows.numel()} [{int(rows[0])}..{int(rows[-1])}] tiles {tiles[:20].tolist()} (n={tiles.numel()}) "
                  f"cols {cols.numel()} [{int(cols[0])}..{int(cols[-1])}] rows%64 {torch.unique(rows % 64)[:32].tolist()}")
