"""ORACLE — test infrastructure only, never the product path.

CPU fp32 restatement of the reference ChunkFormer encoder (ishine/chunkformer,
mounted read-only at /root/reference).  Written from the closed forms in
SURVEY §0.4/§0.5/§A.2-A.3, not by copying the reference.  Only `tests/`,
`__graft_entry__.smoke()` and `bench.py`'s `cpu_baseline` leg may import this
module; the shipped path (`chunkformer_amd`) never does.

Parity pinning: every function is checked against golden fixtures produced by
the reference itself (tests/golden/gen_golden.py imports the reference through
a namespace shim in the build container and records inputs/outputs).

Functions and the reference code they restate:
  plan_utterance / masks_closed_form  encoder.py:534-604 (packer) + 625-645 (masks)
  calc_length                         subsampling.py:270-288
  pos_table                           embedding.py:119-142, 144-174
  frontend                            cmvn.py:32-43, subsampling.py:120-175, embedding.py:176-206
  layer_masked                        encoder_layer.py:155-248, attention.py:420-505,
                                      convolution.py:194-255, positionwise_feed_forward.py:51-60
  forward_parallel_chunk              encoder.py:503-681
  forward_encoder (padded/full)       encoder.py:220-308, encoder_layer.py:62-153,
                                      attention.py:268-418, convolution.py:101-192
  forward_chunk (streaming)           encoder.py:310-385, attention.py:326-333 + 390-418 (cached
                                      branch, rel_shift 242-266), convolution.py:101-192
  ctc_log_softmax                     ctc.py:73-81
"""
from __future__ import annotations

import math
from typing import Dict, List, Optional, Sequence, Tuple

import numpy as np
import torch
import torch.nn.functional as F

SUB = 8          # subsampling rate (encoder.py:138)
CTX = 15         # embed.right_context + 1 (subsampling.py:45, encoder.py:534)
LORDER = 7       # cnn_module_kernel // 2


# ----------------------------------------------------------------------------- integers
def calc_length(T: int) -> int:
    """subsampling.py:270-288: three times floor((L - 3)/2 + 1) in float."""
    L = float(T)
    for _ in range(3):
        L = math.floor((L - 3.0) / 2.0 + 1.0)
    return int(L)


def plan_utterance(T: int, C: int) -> Tuple[int, int]:
    """(n_pad, n_chunk) of one utterance, encoder.py:556-562."""
    size = (C - 1) * SUB + CTX
    step = SUB * C
    if T >= size:
        n_pad = (step - ((T - size) % step)) % step
    else:
        n_pad = size - T
    n_chunk = (T + n_pad - size) // step + 1
    return n_pad, n_chunk


def masks_closed_form(lens: Sequence[int], offsets: Sequence[int], C: int, L: int, R: int):
    """att_mask [N, L+C+R] and mask_pad [N, C+14] (bool) + n_chunks (encoder.py:565-645).

    For utterance u with max_len = 1 + (T_u - 15)//8 and carried offset o_u,
    chunk c (0-based within u) and window index j:
      attention key  g = C*c - L + j : valid iff -o_u <= g < max_len
      conv window    g = C*c - 7 + j : valid iff -o_u <= g < max_len and j-7 <= C+R-1
    """
    att, pad, n_chunks = [], [], []
    for T, o in zip(lens, offsets):
        _, n = plan_utterance(int(T), C)
        max_len = 1 + (int(T) - CTX) // SUB
        c = np.arange(n)[:, None]
        j = np.arange(L + C + R)[None, :]
        g = C * c - L + j
        att.append((g >= -o) & (g < max_len))
        j2 = np.arange(C + 2 * LORDER)[None, :]
        g2 = C * c - LORDER + j2
        pad.append((g2 >= -o) & (g2 < max_len) & (j2 - LORDER <= C + R - 1))
        n_chunks.append(n)
    return np.concatenate(att, 0), np.concatenate(pad, 0), n_chunks


# ----------------------------------------------------------------------------- tables
def pos_table(d: int, max_len: int = 5000) -> torch.Tensor:
    """Relative PE table [2*max_len-1, d]; row r <-> relative distance max_len-1-r."""
    pos = torch.arange(0, max_len, dtype=torch.float32).unsqueeze(1)
    div = torch.exp(torch.arange(0, d, 2, dtype=torch.float32) * -(math.log(10000.0) / d))
    pp = torch.zeros(max_len, d)
    pn = torch.zeros(max_len, d)
    pp[:, 0::2] = torch.sin(pos * div)
    pp[:, 1::2] = torch.cos(pos * div)
    pn[:, 0::2] = torch.sin(-1 * pos * div)
    pn[:, 1::2] = torch.cos(-1 * pos * div)
    return torch.cat([torch.flip(pp, [0]), pn[1:]], 0)


def pos_slice(d: int, C: int, L: int, R: int) -> torch.Tensor:
    """pos_emb rows for window [L, C, R]: L+2C+R-1 rows, row k <-> distance C+L-1-k."""
    pe = pos_table(d)
    ctr = pe.size(0) // 2
    assert L + C < 5000
    return pe[ctr - (C + L) + 1: ctr + C + R]


# ----------------------------------------------------------------------------- modules
def _ln(x, sd, p, eps=1e-5):
    return F.layer_norm(x, (x.size(-1),), sd[p + ".weight"], sd[p + ".bias"], eps)


def _lin(x, sd, p, bias=True):
    return F.linear(x, sd[p + ".weight"], sd[p + ".bias"] if bias else None)


def _ffn(x, sd, p):
    return _lin(F.silu(_lin(x, sd, p + ".w_1")), sd, p + ".w_2")


def frontend(win: torch.Tensor, sd: Dict[str, torch.Tensor], d: int) -> torch.Tensor:
    """[N, W, 80] windows (CMVN already applied) -> [N, T', d] scaled by sqrt(d)."""
    e = "encoder.embed."
    x = win.unsqueeze(1)
    x = F.relu(F.conv2d(x, sd[e + "conv.0.weight"], sd[e + "conv.0.bias"], stride=2))
    for dw, pw in ((2, 3), (5, 6)):
        x = F.conv2d(x, sd[e + f"conv.{dw}.weight"], sd[e + f"conv.{dw}.bias"], stride=2, groups=d)
        x = F.relu(F.conv2d(x, sd[e + f"conv.{pw}.weight"], sd[e + f"conv.{pw}.bias"]))
    n, c, t, f = x.shape
    x = x.permute(0, 2, 1, 3).reshape(n, t, c * f)          # feature index c*F + f
    x = _lin(x, sd, e + "out")
    return x * math.sqrt(d)


def cmvn(x, sd):
    if "encoder.global_cmvn.mean" in sd:
        x = (x - sd["encoder.global_cmvn.mean"]) * sd["encoder.global_cmvn.istd"]
    return x


def _attention_core(q, kw, vw, P, u, v, key_mask, dk, A=None):
    """q [B,Cq,H,dk]; kw/vw [B,W,H,dk]; P [PL,H,dk]; key_mask [B,Cq or 1,W] bool.
    score(i,j) = ((q_i+u).k_j + (q_i+v).P[A-i+j]) / sqrt(dk), A = PL - W by default (= C-1 for
    the chunk window, T'-1 for full attention).  Masked -> -inf, softmax fp32, masked -> 0."""
    B, Cq, H, _ = q.shape
    W = kw.shape[1]
    ac = torch.einsum("bihd,bjhd->bhij", q + u, kw)
    bdf = torch.einsum("bihd,khd->bhik", q + v, P)
    if A is None:
        A = P.shape[0] - W
    idx = A - torch.arange(Cq)[:, None] + torch.arange(W)[None, :]
    bd = torch.gather(bdf, 3, idx.expand(B, H, Cq, W))
    s = (ac + bd) / math.sqrt(dk)
    m = ~key_mask.unsqueeze(1)
    s = s.masked_fill(m, float("-inf"))
    p = torch.softmax(s.float(), dim=-1).masked_fill(m, 0.0)
    return torch.einsum("bhij,bjhd->bihd", p, vw).reshape(B, Cq, H * dk)


def layer_masked(x, sd, p, cfg, att_mask, mask_pad, pos, C, L, R, att_cache, cnn_cache, trunc):
    """One ChunkFormerEncoderLayer.forward_parallel_chunk on x [N, C, d]."""
    N = x.shape[0]
    d, H, dk = cfg.d_model, cfg.n_heads, cfg.head_dim
    x = x + 0.5 * _ffn(_ln(x, sd, p + "norm_ff_macaron"), sd, p + "feed_forward_macaron")
    # ---- MHSA over the overlapping-chunk KV stream
    h = _ln(x, sd, p + "norm_mha")
    a = p + "self_attn."
    q = _lin(h, sd, a + "linear_q").view(N, C, H, dk)
    k = _lin(h, sd, a + "linear_k").view(N * C, H, dk)
    v = _lin(h, sd, a + "linear_v").view(N * C, H, dk)
    cache = att_cache if att_cache is not None else torch.zeros(L, H, 2 * dk)
    flat = torch.cat([cache, torch.cat([k, v], -1)], 0)
    new_att = None
    if att_cache is not None:   # before the right zero padding (attention.py:466-468): a stream shorter than
        new_att = flat[: trunc + L][-L:].clone()   # trunc keeps its last L rows, not padding
    flat = torch.cat([flat, torch.zeros(R, H, 2 * dk)], 0)
    rows = torch.arange(N)[:, None] * C + torch.arange(L + C + R)[None, :]
    win = flat[rows]                                          # [N, W, H, 2dk]
    P = F.linear(pos, sd[a + "linear_pos.weight"]).view(-1, H, dk)
    o = _attention_core(q, win[..., :dk], win[..., dk:], P, sd[a + "pos_bias_u"], sd[a + "pos_bias_v"],
                        att_mask.unsqueeze(1), dk)
    x = x + _lin(o, sd, a + "linear_out")
    # ---- convolution module on the overlapping-chunk GLU stream
    h = _ln(x, sd, p + "norm_conv")
    c = p + "conv_module."
    g = F.linear(h, sd[c + "pointwise_conv1.weight"][:, :, 0], sd[c + "pointwise_conv1.bias"])
    glu = g[..., :d] * torch.sigmoid(g[..., d:])
    cc = cnn_cache.t() if cnn_cache is not None else torch.zeros(LORDER, d)
    flat = torch.cat([cc, glu.reshape(N * C, d)], 0)
    new_cnn = None
    if cnn_cache is not None:   # before the zero padding (convolution.py:228-233)
        new_cnn = flat[: trunc + LORDER][-LORDER:].t().contiguous()
    flat = torch.cat([flat, torch.zeros(LORDER, d)], 0)
    rows = torch.arange(N)[:, None] * C + torch.arange(C + 2 * LORDER)[None, :]
    win = flat[rows] * mask_pad.unsqueeze(-1)                  # [N, C+14, d]
    wdw = sd[c + "depthwise_conv.weight"][:, 0, :]             # [d, 15]
    y = sd[c + "depthwise_conv.bias"].expand(N, C, d).clone()
    for t in range(2 * LORDER + 1):
        y = y + win[:, t: t + C, :] * wdw[:, t]
    y = F.silu(_ln(y, sd, c + "norm"))
    y = F.linear(y, sd[c + "pointwise_conv2.weight"][:, :, 0], sd[c + "pointwise_conv2.bias"])
    y = y * mask_pad[:, LORDER: LORDER + C].unsqueeze(-1)
    x = x + y
    x = x + 0.5 * _ffn(_ln(x, sd, p + "norm_ff"), sd, p + "feed_forward")
    x = _ln(x, sd, p + "norm_final")
    return x, new_att, new_cnn


def pack_windows(xs: List[torch.Tensor], C: int) -> Tuple[torch.Tensor, List[int]]:
    """Per utterance: zero-pad, cut windows of (C-1)*8+15 rows with stride 8C, concat."""
    size = (C - 1) * SUB + CTX
    wins, ns = [], []
    for x in xs:
        T = x.shape[0]
        n_pad, n = plan_utterance(T, C)
        xp = torch.cat([x, torch.zeros(n_pad, x.shape[1])], 0)
        idx = torch.arange(n)[:, None] * (SUB * C) + torch.arange(size)[None, :]
        wins.append(xp[idx])
        ns.append(n)
    return torch.cat(wins, 0), ns


@torch.no_grad()
def forward_parallel_chunk(sd, cfg, xs, lens, C, L, R, att_cache=None, cnn_cache=None,
                           truncated_context_size=0, offset=None):
    """Restatement of ChunkFormerEncoder.forward_parallel_chunk (encoder.py:503-681).

    Returns (out [N,C,d], out_lens [B] int32, n_chunks, att_cache', cnn_cache', offset').
    Caches are the per-layer stacks [nb, L, H, 2dk] / [nb, d, 7] or None."""
    B = len(xs)
    lens = [int(t) for t in lens]
    offs = [0] * B if offset is None else [int(o) for o in offset]
    att_mask, mask_pad, n_chunks = masks_closed_form(lens, offs, C, L, R)
    att_mask = torch.from_numpy(att_mask)
    mask_pad = torch.from_numpy(mask_pad).float()
    win, _ = pack_windows([x.float() for x in xs], C)
    x = frontend(cmvn(win, sd), sd, cfg.d_model)
    pos = pos_slice(cfg.d_model, C, L, R)
    new_att, new_cnn = [], []
    for li in range(cfg.num_blocks):
        x, na, nc = layer_masked(x, sd, f"encoder.encoders.{li}.", cfg, att_mask, mask_pad, pos, C, L, R,
                                 None if att_cache is None else att_cache[li],
                                 None if cnn_cache is None else cnn_cache[li], truncated_context_size)
        new_att.append(na)
        new_cnn.append(nc)
    x = _ln(x, sd, "encoder.after_norm")
    out_lens = torch.tensor([calc_length(t) for t in lens], dtype=torch.int32)
    new_offset = torch.tensor(offs, dtype=torch.int64) + out_lens
    ra = torch.stack(new_att) if att_cache is not None else None
    rc = torch.stack(new_cnn) if cnn_cache is not None else None
    return x, out_lens, n_chunks, ra, rc, new_offset


# ----------------------------------------------------------------------------- padded path
def _attention_padded(h, sd, a, cfg, lens_sub, C, L, R, pos):
    B, T, d = h.shape
    H, dk = cfg.n_heads, cfg.head_dim
    q = _lin(h, sd, a + "linear_q").view(B, T, H, dk)
    k = _lin(h, sd, a + "linear_k").view(B, T, H, dk)
    v = _lin(h, sd, a + "linear_v").view(B, T, H, dk)
    P = F.linear(pos, sd[a + "linear_pos.weight"]).view(-1, H, dk)
    valid = torch.arange(T)[None, :] < lens_sub[:, None]                   # [B, T]
    u, vb = sd[a + "pos_bias_u"], sd[a + "pos_bias_v"]
    if C <= 0:                                                              # full attention
        o = _attention_core(q, k, v, P, u, vb, valid[:, None, :], dk)
        return _lin(o, sd, a + "linear_out")
    n_pad = (C - ((T - C) % C)) % C
    nch = (T + n_pad) // C
    z = lambda t, l, r: torch.cat([torch.zeros(B, l, *t.shape[2:]), t, torch.zeros(B, r, *t.shape[2:])], 1)
    qp = z(q, 0, n_pad).view(B * nch, C, H, dk)
    kp, vp = z(k, L, n_pad + R), z(v, L, n_pad + R)
    rows = torch.arange(nch)[:, None] * C + torch.arange(L + C + R)[None, :]
    kw = kp[:, rows].reshape(B * nch, L + C + R, H, dk)
    vw = vp[:, rows].reshape(B * nch, L + C + R, H, dk)
    vq = torch.cat([valid, torch.zeros(B, n_pad, dtype=torch.bool)], 1).view(B * nch, C)
    vk = torch.cat([torch.zeros(B, L, dtype=torch.bool), valid, torch.zeros(B, n_pad + R, dtype=torch.bool)], 1)
    vk = vk[:, rows].reshape(B * nch, L + C + R)
    mask = vq[:, :, None] & vk[:, None, :]
    o = _attention_core(qp, kw, vw, P, u, vb, mask, dk)
    o = _lin(o, sd, a + "linear_out").view(B, nch * C, d)
    return o[:, :T]


def _conv_padded(h, sd, c, cfg, lens_sub, C):
    B, T, d = h.shape
    valid = (torch.arange(T)[None, :] < lens_sub[:, None]).float().unsqueeze(-1)
    g = F.linear(h * valid, sd[c + "pointwise_conv1.weight"][:, :, 0], sd[c + "pointwise_conv1.bias"])
    glu = g[..., :d] * torch.sigmoid(g[..., d:])                           # [B, T, d]
    Ce = T if C <= 0 else C
    t = torch.arange(T)
    chunk_lo = (t // Ce) * Ce - LORDER                                     # left context is real
    chunk_hi = (t // Ce) * Ce + Ce                                         # right context zero-padded
    wdw = sd[c + "depthwise_conv.weight"][:, 0, :]
    y = sd[c + "depthwise_conv.bias"].expand(B, T, d).clone()
    for tap in range(2 * LORDER + 1):
        src = t + tap - LORDER
        ok = (src >= 0) & (src >= chunk_lo) & (src < chunk_hi) & (src < T)
        vals = glu[:, src.clamp(0, T - 1)] * ok.float()[None, :, None]
        y = y + vals * wdw[:, tap]
    y = F.silu(_ln(y, sd, c + "norm"))
    y = F.linear(y, sd[c + "pointwise_conv2.weight"][:, :, 0], sd[c + "pointwise_conv2.bias"])
    return y * valid


@torch.no_grad()
def forward_encoder(sd, cfg, xs, xs_lens, C=0, L=0, R=0):
    """Restatement of ChunkFormerEncoder.forward_encoder (encoder.py:220-274): padded batch
    [B, T, 80] -> ([B, T', d], masks [B, 1, T'] bool).  C<=0 -> full attention."""
    B, T, _ = xs.shape
    x = cmvn(xs.float(), sd)
    x = frontend(x, sd, cfg.d_model)
    Tp = x.shape[1]
    lens_sub = torch.tensor([max(calc_length(int(t)), -1) for t in xs_lens])
    Ce = Tp if C <= 0 else C
    Le, Re = (0, 0) if C <= 0 else (L, R)
    pos = pos_slice(cfg.d_model, Ce, Le, Re)
    for li in range(cfg.num_blocks):
        p = f"encoder.encoders.{li}."
        x = x + 0.5 * _ffn(_ln(x, sd, p + "norm_ff_macaron"), sd, p + "feed_forward_macaron")
        x = x + _attention_padded(_ln(x, sd, p + "norm_mha"), sd, p + "self_attn.", cfg, lens_sub, C, Le, Re, pos)
        x = x + _conv_padded(_ln(x, sd, p + "norm_conv"), sd, p + "conv_module.", cfg, lens_sub, C)
        x = x + 0.5 * _ffn(_ln(x, sd, p + "norm_ff"), sd, p + "feed_forward")
        x = _ln(x, sd, p + "norm_final")
    x = _ln(x, sd, "encoder.after_norm")
    masks = (torch.arange(Tp)[None, :] < lens_sub[:, None]).unsqueeze(1)
    return x, masks


@torch.no_grad()
def forward_chunk(sd, cfg, xs, att_cache, cnn_cache, C, L, R, offset):
    """Restatement of ChunkFormerEncoder.forward_chunk (encoder.py:310-385), the realtime path:
    xs [B, T, 80] (no padding), att_cache [nb, B, H, L, 2dk], cnn_cache [nb, B, d, 7], integer
    offset.  Returns (xs [B, T', d], new att_cache [nb, B, H, L, 2dk], new cnn_cache [nb, B, d, 7]).

    Per layer (chunk_size C, right context 0): every one of the T' queries attends to the L cached
    keys + the T' current keys; key j is valid iff j >= L - offset (the flipped att_masks of
    encoder.py:351-357, cut to L + T' keys, attention.py:132); the rel-pos table is the one of a
    chunk of C + R frames (embed called with chunk_size = C + R, encoder.py:343-349) read by
    rel_shift with time1 = T' (row T'-1-i+j, attention.py:256-266).  The conv module concatenates
    the 7-frame cache and runs the dynamic chunk conv at chunk size C (convolution.py:133-180).
    New caches: the L keys/values and the 7 GLU frames ending R frames before the chunk end
    (encoder.py:374-383)."""
    B, T, _ = xs.shape
    d, H, dk = cfg.d_model, cfg.n_heads, cfg.head_dim
    x = frontend(cmvn(xs.float(), sd), sd, d)                       # [B, T', d]
    Tp = x.shape[1]
    assert Tp >= R, "forward_chunk needs T' >= right_context_size (cache slicing)"
    pos = pos_slice(d, C + R, L, 0)
    key_valid = (torch.arange(L + Tp) >= L - int(offset))[None, None, :].expand(B, 1, L + Tp)
    new_att, new_cnn = [], []
    for li in range(cfg.num_blocks):
        p = f"encoder.encoders.{li}."
        x = x + 0.5 * _ffn(_ln(x, sd, p + "norm_ff_macaron"), sd, p + "feed_forward_macaron")
        h = _ln(x, sd, p + "norm_mha")
        a = p + "self_attn."
        q = _lin(h, sd, a + "linear_q").view(B, Tp, H, dk)
        k = _lin(h, sd, a + "linear_k").view(B, Tp, H, dk)
        v = _lin(h, sd, a + "linear_v").view(B, Tp, H, dk)
        cache = att_cache[li].permute(0, 2, 1, 3).float()           # [B, L, H, 2dk]
        kv = torch.cat([cache, torch.cat([k, v], -1)], 1)             # [B, L + T', H, 2dk]
        new_att.append(kv[:, Tp - R: Tp - R + L].permute(0, 2, 1, 3).clone())
        P = F.linear(pos, sd[a + "linear_pos.weight"]).view(-1, H, dk)
        o = _attention_core(q, kv[..., :dk], kv[..., dk:], P, sd[a + "pos_bias_u"], sd[a + "pos_bias_v"],
                            key_valid, dk, A=Tp - 1)
        x = x + _lin(o, sd, a + "linear_out")
        h = _ln(x, sd, p + "norm_conv")
        c = p + "conv_module."
        g = F.linear(h, sd[c + "pointwise_conv1.weight"][:, :, 0], sd[c + "pointwise_conv1.bias"])
        glu = g[..., :d] * torch.sigmoid(g[..., d:])
        xc = torch.cat([cnn_cache[li].transpose(1, 2).float(), glu], 1)   # [B, 7 + T', d]
        new_cnn.append(xc[:, Tp - R: Tp - R + LORDER].transpose(1, 2).clone())
        wdw = sd[c + "depthwise_conv.weight"][:, 0, :]
        y = sd[c + "depthwise_conv.bias"].expand(B, Tp, d).clone()
        t = torch.arange(Tp)
        lim = torch.clamp((t // C) * C + C + LORDER, max=LORDER + Tp)      # chunk end / sequence end
        for tap in range(2 * LORDER + 1):
            src = t + tap                                                  # index into xc
            ok = (src < lim).float()[None, :, None]
            y = y + xc[:, src.clamp(max=LORDER + Tp - 1)] * ok * wdw[:, tap]
        y = F.silu(_ln(y, sd, c + "norm"))
        y = F.linear(y, sd[c + "pointwise_conv2.weight"][:, :, 0], sd[c + "pointwise_conv2.bias"])
        x = x + y
        x = x + 0.5 * _ffn(_ln(x, sd, p + "norm_ff"), sd, p + "feed_forward")
        x = _ln(x, sd, p + "norm_final")
    x = _ln(x, sd, "encoder.after_norm")
    return x, torch.stack(new_att), torch.stack(new_cnn)


@torch.no_grad()
def ctc_log_softmax(sd, enc):
    """ctc.py:73-81."""
    return F.log_softmax(F.linear(enc, sd["ctc.ctc_lo.weight"], sd["ctc.ctc_lo.bias"]), dim=-1)


@torch.no_grad()
def forward_chunk_by_chunk(sd, cfg, xs, xs_lens, C, L, R):
    """Restatement of ChunkFormerEncoder.forward_chunk_by_chunk (encoder.py:387-459): xs [B, T, 80] padded by
    stride - ((T - size) % stride) zero frames (size = 8 (C - 1) + 15 + 8 R input frames per step, the
    reverse of calc_length, subsampling.py:290-311; stride 8 C), then forward_chunk per step with the caches
    carried and offset += C; every step keeps its first C rows but the last one its whole output.  Returns
    (out [B, T', d], masks [B, 1, max calc_length(xs_lens + pad)])."""
    B = xs.shape[0]
    nb, H, dk, d = cfg.num_blocks, cfg.n_heads, cfg.head_dim, cfg.d_model
    size = 8 * (C - 1) + 15 + 8 * R
    stride = 8 * C
    pad = stride - ((xs.shape[1] - size) % stride)
    xs = torch.nn.functional.pad(xs.float(), (0, 0, 0, pad))
    lens = [int(t) + pad for t in xs_lens]
    att = torch.zeros(nb, B, H, L, 2 * dk)
    cnn = torch.zeros(nb, B, d, 7)
    outs, offset = [], 0
    for i in range(0, xs.shape[1] - size + stride, stride):
        y, att, cnn = forward_chunk(sd, cfg, xs[:, i: i + size], att, cnn, C, L, R, offset)
        outs.append(y[:, :C] if i + size < xs.shape[1] else y)
        offset += C
    sub = torch.tensor([calc_length(t) for t in lens])
    masks = (torch.arange(int(sub.max()))[None, :] < sub[:, None]).unsqueeze(1)
    return torch.cat(outs, 1), masks
