"""State-dict schema of the reference encoder + a deterministic synthetic recipe.

Key names and shapes follow the reference module tree:
  * front-end   `chunkformer/modules/subsampling.py:69-112` (embed.conv.{0,2,3,5,6}, embed.out)
  * CMVN        `chunkformer/modules/cmvn.py:22-30` (global_cmvn.mean / istd)
  * per layer   `chunkformer/modules/encoder_layer.py:29-60`, `attention.py:230-240`,
                `convolution.py:48-98`, `positionwise_feed_forward.py:46-49`
  * tail        `encoder.py:119` (after_norm), `ctc.py:47` (ctc.ctc_lo)

No checkpoint is reachable offline, so weights come from `synthetic_state_dict`,
a seeded recipe with the reference's default init magnitudes (U(-1/sqrt(fan_in),
+1/sqrt(fan_in)) for linear/conv, xavier-uniform for pos_bias_u/v, LayerNorm
weight 1 +- 0.05).  It runs on the CPU RNG, so the same seed gives the same
weights here and on the GPU box.
"""
from __future__ import annotations

import math
from collections import OrderedDict
from typing import Dict, List, Tuple

import torch

from .config import EncoderConfig

ENC = "encoder."


def schema(cfg: EncoderConfig) -> List[Tuple[str, Tuple[int, ...]]]:
    """Ordered (name, shape) list of every tensor the encoder (+CTC) needs."""
    d, ff, h, dk, k = cfg.d_model, cfg.ffn_dim, cfg.n_heads, cfg.head_dim, cfg.kernel_size
    out: List[Tuple[str, Tuple[int, ...]]] = []
    if cfg.cmvn:
        out += [(ENC + "global_cmvn.mean", (cfg.input_dim,)), (ENC + "global_cmvn.istd", (cfg.input_dim,))]
    e = ENC + "embed."
    out += [(e + "conv.0.weight", (d, 1, 3, 3)), (e + "conv.0.bias", (d,))]
    for i in (2, 5):   # depthwise 3x3 s2
        out += [(e + f"conv.{i}.weight", (d, 1, 3, 3)), (e + f"conv.{i}.bias", (d,))]
    for i in (3, 6):   # pointwise 1x1
        out += [(e + f"conv.{i}.weight", (d, d, 1, 1)), (e + f"conv.{i}.bias", (d,))]
    f_out = ((cfg.input_dim - 1) // 2 - 1) // 2
    f_out = (f_out - 1) // 2                      # 80 -> 39 -> 19 -> 9
    out += [(e + "out.weight", (d, d * f_out)), (e + "out.bias", (d,))]
    for li in range(cfg.num_blocks):
        p = ENC + f"encoders.{li}."
        for ffn in ("feed_forward_macaron", "feed_forward"):
            out += [(p + ffn + ".w_1.weight", (ff, d)), (p + ffn + ".w_1.bias", (ff,)),
                    (p + ffn + ".w_2.weight", (d, ff)), (p + ffn + ".w_2.bias", (d,))]
        a = p + "self_attn."
        for nm in ("linear_q", "linear_k", "linear_v", "linear_out"):
            out += [(a + nm + ".weight", (d, d)), (a + nm + ".bias", (d,))]
        out += [(a + "linear_pos.weight", (d, d)), (a + "pos_bias_u", (h, dk)), (a + "pos_bias_v", (h, dk))]
        c = p + "conv_module."
        out += [(c + "pointwise_conv1.weight", (2 * d, d, 1)), (c + "pointwise_conv1.bias", (2 * d,)),
                (c + "depthwise_conv.weight", (d, 1, k)), (c + "depthwise_conv.bias", (d,)),
                (c + "norm.weight", (d,)), (c + "norm.bias", (d,)),
                (c + "pointwise_conv2.weight", (d, d, 1)), (c + "pointwise_conv2.bias", (d,))]
        for nm in ("norm_ff", "norm_mha", "norm_ff_macaron", "norm_conv", "norm_final"):
            out += [(p + nm + ".weight", (d,)), (p + nm + ".bias", (d,))]
    out += [(ENC + "after_norm.weight", (d,)), (ENC + "after_norm.bias", (d,))]
    if cfg.vocab > 0:
        out += [("ctc.ctc_lo.weight", (cfg.vocab, d)), ("ctc.ctc_lo.bias", (cfg.vocab,))]
    return out


def _fan_in(name: str, shape: Tuple[int, ...]) -> int:
    if len(shape) == 1:
        return 0
    return int(math.prod(shape[1:]))


def synthetic_state_dict(cfg: EncoderConfig, seed: int = 0) -> "OrderedDict[str, torch.Tensor]":
    """Deterministic random weights with the reference's init magnitudes."""
    g = torch.Generator().manual_seed(seed)
    sd: "OrderedDict[str, torch.Tensor]" = OrderedDict()
    shapes = dict(schema(cfg))

    def U(shape, a):
        return (torch.rand(shape, generator=g, dtype=torch.float32) * 2.0 - 1.0) * a

    for name, shape in schema(cfg):
        if name.endswith("global_cmvn.mean"):
            t = U(shape, 0.5)
        elif name.endswith("global_cmvn.istd"):
            t = 1.0 + U(shape, 0.5)
        elif name.endswith("pos_bias_u") or name.endswith("pos_bias_v"):
            t = U(shape, math.sqrt(6.0 / (shape[0] + shape[1])))
        elif ("norm" in name.split(".")[-2] or name.split(".")[-2].startswith("norm")) and len(shape) == 1:
            t = (1.0 + U(shape, 0.05)) if name.endswith("weight") else U(shape, 0.05)
        elif name.endswith("bias"):
            wshape = shapes[name[: -len("bias")] + "weight"]
            t = U(shape, 1.0 / math.sqrt(_fan_in(name, wshape)))
        else:
            t = U(shape, 1.0 / math.sqrt(_fan_in(name, shape)))
        sd[name] = t.contiguous()
    return sd


def check_state_dict(cfg: EncoderConfig, sd: Dict[str, torch.Tensor]) -> None:
    """Raise if a required key is missing or mis-shaped (load_checkpoint is
    strict=False in the reference, checkpoint.py:26-41, but the kernels need
    every tensor)."""
    for name, shape in schema(cfg):
        if name not in sd:
            raise KeyError(f"missing weight {name}")
        if tuple(sd[name].shape) != tuple(shape):
            raise ValueError(f"weight {name}: shape {tuple(sd[name].shape)} != {shape}")


def synthetic_features(lens, seed: int):
    """List of [T_i, 80] N(0,1) fbank-like features from a seeded CPU generator
    (BASELINE.md §3 synthetic inputs)."""
    g = torch.Generator().manual_seed(seed)
    return [torch.randn(int(t), 80, generator=g) for t in lens]


def synthetic_vocab(V: int) -> Dict[int, str]:
    """Deterministic `vocab.txt` stand-in (no real vocabulary is reachable offline): id 0 is
    <blank>, id 1 <unk>, the rest short letter strings, every 5th a word start ('▁' prefix, turned
    into a space by class2str, model_utils.py:135-139)."""
    out = {0: "<blank>", 1: "<unk>"}
    letters = "abcdefghijklmnopqrstuvwxyz"
    for i in range(2, V):
        s, n = "", i
        while True:
            s = letters[n % 26] + s
            n //= 26
            if n == 0:
                break
        out[i] = ("▁" + s) if i % 5 == 0 else s
    return out
