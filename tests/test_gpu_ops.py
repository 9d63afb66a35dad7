"""Kernel-level GPU parity: the projection GEMM (every epilogue, every tile path, bf16, fp16
and exact-f32) against a torch fp32 reference of the same op (cfm_op_gemm, include/cfm_ops.h)."""
import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def L():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from chunkformer_amd import _lib
    return _lib


def _run(L, dtype, epi, act, A, W, bias, alpha=1.0, out=None, ldo=0, row_off=0, out2=None, d=0, x=None,
         rowmask=None, small=0):
    M, K = A.shape
    N = W.shape[0]
    st = torch.cuda.current_stream().cuda_stream
    L.check(L.cfm_op_gemm(dtype, epi, act, A.data_ptr(), K, W.data_ptr(), K, M, N, K, L.ptr(bias), alpha,
                          L.ptr(out), ldo, row_off, L.ptr(out2), d, L.ptr(x), N if x is not None else 0,
                          L.ptr(rowmask), small, st))
    torch.cuda.synchronize()


def _ref(A, W, bias):
    r = A.float() @ W.float().t()
    return r + bias if bias is not None else r


def _close(got, exp, tol):
    err = (got.float() - exp).abs().max().item()
    scale = exp.abs().max().item() + 1e-6
    assert err <= tol * scale, f"max err {err} vs scale {scale}"


SHAPES = [(1000, 512, 512), (700, 2048, 512), (513, 512, 2048), (256, 256, 4608), (300, 48, 128),
          (70001, 512, 2048), (2000, 512, 4608), (129, 512, 1024),   # N = 512, K >= 1024 (FFN w2, front-end out)
          (70001, 512, 512), (33000, 2048, 512),   # these two run the K = 512 weight-in-registers kernel
          (40000, 1536, 512),
          (1000, 256, 128), (4097, 768, 384)]      # shortest ring K (4 steps); K % 128 != 0 (K-64 kernel)
# variant bits (include/cfm_ops.h): 1 = 128x128 tiles; 7 << 18 = K = 512 weight-stationary kernel off
# (the 256 x 256 kernel takes its shapes); 2 << 16 = nt stores
MODES = [("bf16", 0), ("bf16", 1), ("fp32", 0), ("bf16", 7 << 18), ("bf16", 2 << 16),
         ("fp16", 0), ("fp16", 1), ("fp16", 7 << 18)]   # fp16: the same kernels on f16 MFMA (EpiArgs::f16)


def _dt(L, dt):
    """(torch dtype, cfm_dtype code, max-error tolerance relative to the output scale)"""
    return {"bf16": (torch.bfloat16, L.DTYPE_BF16, 1e-2), "fp16": (torch.float16, L.DTYPE_F16, 2e-3),
            "fp32": (torch.float32, L.DTYPE_F32, 1e-5)}[dt]


@pytest.mark.parametrize("M,N,K", SHAPES)
@pytest.mark.parametrize("mode", MODES)
@pytest.mark.parametrize("act", [0, 1, 2, 3])   # 3: SiLU on a -log2(e)-prescaled input (a / (1 + 2^a))
def test_gemm_store(L, M, N, K, mode, act):
    dt, small = mode
    tdt, code, tol = _dt(L, dt)
    g = torch.Generator(device="cuda").manual_seed(M + N + K)
    A = (torch.randn(M, K, device="cuda", generator=g) * 0.5).to(tdt)
    W = (torch.randn(N, K, device="cuda", generator=g) / K ** 0.5).to(tdt)
    bias = torch.randn(N, device="cuda", generator=g)
    out = torch.full((M + 3, N), float("nan"), device="cuda", dtype=tdt)
    _run(L, code, 0, act, A, W, bias, out=out, ldo=N, row_off=3, small=small)
    r = _ref(A, W, bias)
    r = torch.relu(r) if act == 1 else (torch.nn.functional.silu(r) if act == 2 else r)
    if act == 3:
        r = r / (1 + torch.exp2(r))
    _close(out[3:], r, tol)
    assert torch.isnan(out[:3].float()).all()


@pytest.mark.parametrize("M,N,K", [(70001, 512, 512), (1000, 256, 4608)])
def test_gemm_no_bias(L, M, N, K):
    g = torch.Generator(device="cuda").manual_seed(7)
    A = (torch.randn(M, K, device="cuda", generator=g) * 0.5).to(torch.bfloat16)
    W = (torch.randn(N, K, device="cuda", generator=g) / K ** 0.5).to(torch.bfloat16)
    out = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
    _run(L, L.DTYPE_BF16, 0, 0, A, W, None, out=out, ldo=N)
    _close(out, _ref(A, W, None), 1e-2)


@pytest.mark.parametrize("mode", MODES)
def test_gemm_store_f32_and_resid(L, mode):
    dt, small = mode
    tdt, code, _ = _dt(L, dt)
    M, N, K = 777, 512, 4608
    g = torch.Generator(device="cuda").manual_seed(5)
    A = (torch.randn(M, K, device="cuda", generator=g) * 0.5).to(tdt)
    W = (torch.randn(N, K, device="cuda", generator=g) / K ** 0.5).to(tdt)
    bias = torch.randn(N, device="cuda", generator=g)
    out = torch.empty(M, N, device="cuda")
    _run(L, code, 1, 0, A, W, bias, alpha=22.627, out=out, ldo=N, small=small)
    _close(out, 22.627 * _ref(A, W, bias), 1e-5 if dt == "fp32" else 1e-3)
    x0 = torch.randn(M, N, device="cuda", generator=g)
    x = x0.clone()
    rm = (torch.rand(M, device="cuda", generator=g) > 0.3).to(torch.uint8)
    _run(L, code, 2, 0, A, W, bias, alpha=0.5, x=x, rowmask=rm, small=small)
    _close(x, x0 + 0.5 * _ref(A, W, bias) * rm.float()[:, None], 1e-5 if dt == "fp32" else 1e-3)


@pytest.mark.parametrize("mode", MODES)
@pytest.mark.parametrize("M", [900, 40000])   # 40000 rows: the K = 512 weight-in-registers kernel
def test_gemm_qkv_and_glu(L, mode, M):
    dt, small = mode
    tdt, code, tol = _dt(L, dt)
    d, Lc = 512, 5
    g = torch.Generator(device="cuda").manual_seed(9)
    A = (torch.randn(M, d, device="cuda", generator=g) * 0.5).to(tdt)
    W = (torch.randn(3 * d, d, device="cuda", generator=g) / d ** 0.5).to(tdt)
    bias = torch.randn(3 * d, device="cuda", generator=g)
    q = torch.empty(M, d, device="cuda", dtype=tdt)
    kv = torch.zeros(M + Lc + 2, 2 * d, device="cuda", dtype=tdt)
    _run(L, code, 3, 0, A, W, bias, out=q, out2=kv, row_off=Lc, d=d, small=small)
    r = _ref(A, W, bias)
    _close(q, r[:, :d], tol)
    kvr = kv[Lc: Lc + M].view(M, d // 64, 2, 64)
    _close(kvr[:, :, 0].reshape(M, d), r[:, d: 2 * d], tol)
    _close(kvr[:, :, 1].reshape(M, d), r[:, 2 * d:], tol)
    assert (kv[:Lc] == 0).all() and (kv[Lc + M:] == 0).all()
    # GLU with [a16 | gate16] interleaved weights
    W1 = (torch.randn(2 * d, d, device="cuda", generator=g) / d ** 0.5).to(tdt)
    b1 = torch.randn(2 * d, device="cuda", generator=g)
    idx = torch.arange(2 * d, device="cuda").view(d // 16, 2, 16)
    perm = torch.stack([idx[:, 0] // 2 * 0 + torch.arange(d // 16, device="cuda")[:, None] * 16
                        + torch.arange(16, device="cuda")[None, :],
                        d + torch.arange(d // 16, device="cuda")[:, None] * 16 + torch.arange(16, device="cuda")[None, :]],
                       1).reshape(-1)
    out = torch.empty(M + 7, d, device="cuda", dtype=tdt)
    _run(L, code, 4, 0, A, W1[perm].contiguous(), b1[perm].contiguous(), out=out, ldo=d, row_off=7, small=small)
    r = _ref(A, W1, b1)
    _close(out[7:], r[:, :d] * torch.sigmoid(r[:, d:]), tol)
    # act 3: the gate half arrives pre-scaled by -log2(e) (the model's 16-bit weights): lin / (1 + 2^gate)
    _run(L, code, 4, 3, A, W1[perm].contiguous(), b1[perm].contiguous(), out=out, ldo=d, row_off=7, small=small)
    _close(out[7:], r[:, :d] / (1 + torch.exp2(r[:, d:])), tol)



def test_gemm_output_past_2gib(L):
    """K = 512 weight-stationary kernel with a > 2 GiB output (a 980-minute batch's FFN hidden):
    sampled rows against torch, including the last tile."""
    M, N, K = 540_037, 2048, 512
    g = torch.Generator(device="cuda").manual_seed(11)
    A = (torch.randn(M, K, device="cuda", generator=g) * 0.5).to(torch.bfloat16)
    W = (torch.randn(N, K, device="cuda", generator=g) / K ** 0.5).to(torch.bfloat16)
    bias = torch.randn(N, device="cuda", generator=g)
    out = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
    assert out.numel() * 2 > 2 ** 31
    _run(L, L.DTYPE_BF16, 0, 2, A, W, bias, out=out, ldo=N)
    rows = torch.cat([torch.arange(0, 64), torch.randint(0, M, (2000,), generator=torch.Generator().manual_seed(1)),
                      torch.arange(M - 100, M)]).cuda()
    r = torch.nn.functional.silu(_ref(A[rows], W, bias))
    _close(out[rows], r, 1e-2)
