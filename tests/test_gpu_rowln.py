"""Kernel-level GPU parity of the row-owning GEMM with the residual add and LayerNorm(s) in its
epilogue (cfm_op_gemm_rowln, include/cfm_ops.h; gemm_rowln.hip) against a torch fp32 reference of the
same op: each of the four sub-block sites of an encoder layer (encoder_layer.py:155-248), ragged row
counts, the padded path's row masks, the last layer's f32 after_norm output."""
import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def L():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from chunkformer_amd import _lib
    return _lib


def _ln(x, w, b, eps=1e-5):
    return torch.nn.functional.layer_norm(x, (x.shape[-1],), w, b, eps)


def _ref(A, W, bias, alpha, accmask, x, y1, a1, y1mask, g1, b1, g2, b2, hmask):
    v = (A.float() @ W.float().t() + bias).to(torch.bfloat16).float()
    xn = x.clone()
    if y1 is not None:
        m1 = y1mask.float()[:, None] if y1mask is not None else 1.0
        xn = xn + a1 * m1 * y1.float()
    ma = accmask.float()[:, None] if accmask is not None else 1.0
    xn = xn + alpha * ma * v
    if g2 is None:
        x_out, z = xn, _ln(xn, g1, b1)
    else:
        x_out = _ln(xn, g1, b1)
        z = _ln(x_out, g2, b2)
    if hmask is not None:
        z = z * hmask.float()[:, None]
    return v, x_out, z


SITES = {
    # name: (y_out, y1, x_out, two LNs, f32 out, masks)
    "ffn_mac": dict(y_out=True),
    "linear_out": dict(y1=True, x_out=True, hmask=True),
    "conv_pw2": dict(y_out=True, accmask=True),
    "ffn_final": dict(y1=True, y1mask=True, x_out=True, ln2=True),
    "ffn_last": dict(y1=True, y1mask=True, ln2=True, f_out=True),
}


@pytest.mark.parametrize("site", list(SITES))
@pytest.mark.parametrize("M,K", [(1000, 2048), (300, 512), (70001, 512), (33000, 2048), (128, 512), (40000, 1024)])
def test_rowln_sites(L, site, M, K):
    cfg = SITES[site]
    N = 512
    dev = "cuda"
    g = torch.Generator(device=dev).manual_seed(M + K + len(site))
    A = (torch.randn(M, K, device=dev, generator=g) * 0.5).to(torch.bfloat16)
    W = (torch.randn(N, K, device=dev, generator=g) / K ** 0.5).to(torch.bfloat16)
    bias = torch.randn(N, device=dev, generator=g) * 0.1
    x = torch.randn(M, N, device=dev, generator=g) * 2.0 + 0.3
    y1 = (torch.randn(M, N, device=dev, generator=g)).to(torch.bfloat16) if cfg.get("y1") else None
    rowmask = (torch.rand(M, device=dev, generator=g) > 0.1).to(torch.uint8)
    accmask = rowmask if cfg.get("accmask") else None
    y1mask = rowmask if cfg.get("y1mask") else None
    hmask = rowmask if cfg.get("hmask") else None
    g1, b1 = 1 + 0.1 * torch.randn(N, device=dev, generator=g), 0.1 * torch.randn(N, device=dev, generator=g)
    g2 = b2 = None
    if cfg.get("ln2"):
        g2, b2 = 1 + 0.1 * torch.randn(N, device=dev, generator=g), 0.1 * torch.randn(N, device=dev, generator=g)
    alpha, a1 = 0.5, 0.5 if site == "linear_out" else 1.0
    v_r, x_r, z_r = _ref(A, W, bias, alpha, accmask, x, y1, a1, y1mask, g1, b1, g2, b2, hmask)

    x_in = x.clone()
    y_out = torch.full((M, N), float("nan"), device=dev, dtype=torch.bfloat16) if cfg.get("y_out") else None
    x_out = x_in if cfg.get("x_out") else None   # in place, as the encoder runs it
    h_out = None if cfg.get("f_out") else torch.full((M, N), float("nan"), device=dev, dtype=torch.bfloat16)
    f_out = torch.full((M, N), float("nan"), device=dev) if cfg.get("f_out") else None
    ybuf = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
    st = torch.cuda.current_stream().cuda_stream
    L.check(L.cfm_op_gemm_rowln(A.data_ptr(), K, W.data_ptr(), K, M, K, bias.data_ptr(), alpha, L.ptr(accmask),
                                x_in.data_ptr(), L.ptr(y1), a1, L.ptr(y1mask), L.ptr(y_out), L.ptr(x_out),
                                g1.data_ptr(), b1.data_ptr(), L.ptr(g2), L.ptr(b2), L.ptr(h_out), L.ptr(f_out),
                                L.ptr(hmask), ybuf.data_ptr(), 1e-5, 0, st))
    torch.cuda.synchronize()
    if y_out is not None:   # one bf16 ulp where the f32 sums straddle a rounding boundary
        assert ((y_out.float() - v_r).abs() <= v_r.abs() * 2 ** -7 + 1e-6).all()
    if x_out is not None:
        err = (x_in - x_r).abs().max().item()
        assert err <= 2e-2 * x_r.abs().max().item(), err
    else:
        assert torch.equal(x_in, x), "x must stay untouched without x_out"
    z = f_out if f_out is not None else h_out.float()
    assert not torch.isnan(z).any()
    err = (z - z_r).abs().max().item()
    assert err <= 3e-2, f"LayerNorm output max err {err}"
    rel = ((z - z_r).norm() / z_r.norm()).item()
    assert rel <= 5e-3, rel


def test_ln_fuse_option_matches_layernorm_kernels(L):
    """The whole encoder with the fused sites (model option ln_fuse, off by default) against the LayerNorm
    kernels: masked batch (chunked) and padded full-attention path, 12 layers, bf16."""
    from chunkformer_amd.config import LARGE
    from chunkformer_amd.encoder import ChunkFormerEncoder
    from chunkformer_amd.weights import synthetic_features, synthetic_state_dict
    enc = ChunkFormerEncoder(LARGE, synthetic_state_dict(LARGE, 0), dtype="bf16")
    lens = [1900, 640, 77, 3001]
    xs = synthetic_features(lens, 5)
    outs = {}
    for f in (0, 1):
        enc.set_option("ln_fuse", f)
        o, ol, n, _, _, _ = enc.forward_parallel_chunk(xs, torch.tensor(lens, dtype=torch.int32), 64, 128, 128)
        xp = torch.nn.utils.rnn.pad_sequence(xs, batch_first=True)
        p, pl = enc.forward_encoder(xp, torch.tensor(lens), -1, -1, -1)[:2]
        torch.cuda.synchronize()
        outs[f] = (o.float().cpu(), p.float().cpu())
    enc.set_option("ln_fuse", 0)
    for a, b in zip(outs[0], outs[1]):
        rel = ((a - b).norm() / a.norm()).item()
        assert rel < 1e-2, rel
