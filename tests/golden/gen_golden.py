"""Generate the committed golden fixtures from the REFERENCE implementation.

Runs only in the build container (it imports /root/reference through a namespace
shim: chunkformer/__init__.py pulls audio deps that are absent, the modules we
need import with torch alone).  Nothing on the GPU box reads /root/reference;
the fixtures written here are plain .npz data (inputs + expected outputs).

    python tests/golden/gen_golden.py            # rewrites tests/golden/*.npz

Weights: `chunkformer_amd.weights.synthetic_state_dict(cfg, seed)` (seeded CPU
RNG), loaded into the reference modules with strict=True.
"""
from __future__ import annotations

import os
import sys
import types

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)
sys.dont_write_bytecode = True

REF = "/root/reference/chunkformer"
m = types.ModuleType("chunkformer")
m.__path__ = [REF]
sys.modules["chunkformer"] = m

from chunkformer.modules.cmvn import GlobalCMVN  # noqa: E402
from chunkformer.modules.ctc import CTC  # noqa: E402
from chunkformer.modules.encoder import ChunkFormerEncoder  # noqa: E402

from chunkformer_amd.config import LARGE, SMALL, EncoderConfig  # noqa: E402
from chunkformer_amd.weights import synthetic_features, synthetic_state_dict  # noqa: E402

torch.set_num_threads(8)


def build_reference(cfg: EncoderConfig, seed: int):
    sd = synthetic_state_dict(cfg, seed)
    cmvn = GlobalCMVN(torch.zeros(cfg.input_dim), torch.ones(cfg.input_dim)) if cfg.cmvn else None
    enc = ChunkFormerEncoder(cfg.input_dim, output_size=cfg.d_model, attention_heads=cfg.n_heads,
                             linear_units=cfg.ffn_dim, num_blocks=cfg.num_blocks,
                             cnn_module_kernel=cfg.kernel_size, cnn_module_norm="layer_norm",
                             dynamic_conv=True, activation_type="swish", global_cmvn=cmvn).eval()
    esd = {k[len("encoder."):]: v for k, v in sd.items() if k.startswith("encoder.")}
    enc.load_state_dict(esd, strict=True)
    ctc = None
    if cfg.vocab:
        ctc = CTC(cfg.vocab, cfg.d_model).eval()
        ctc.ctc_lo.weight.data.copy_(sd["ctc.ctc_lo.weight"])
        ctc.ctc_lo.bias.data.copy_(sd["ctc.ctc_lo.bias"])
    return enc, ctc, sd


def feats(lens, seed):
    return synthetic_features(lens, seed)


def sd_digest(sd):
    return np.array([float(v.double().sum()) for v in sd.values()], dtype=np.float64)


# ---------------------------------------------------------------------------- masks
def gen_masks(path):
    """~120 random packer cases; the masks are captured from the first layer call."""
    cfg = EncoderConfig(d_model=64, n_heads=1, ffn_dim=64, num_blocks=1, vocab=0, cmvn=False)
    enc, _, _ = build_reference(cfg, 0)
    cap = {}
    orig = enc.encoders[0].forward_parallel_chunk

    def hook(x, mask, pos_emb, mask_pad, **kw):
        cap["att"], cap["pad"] = mask.clone(), mask_pad.clone()
        return orig(x, mask, pos_emb, mask_pad, **kw)

    enc.encoders[0].forward_parallel_chunk = hook
    rng = np.random.default_rng(1234)
    out = {}
    cases = []
    for i in range(120):
        C = int(rng.choice([1, 2, 4, 8, 16, 64]))
        L = int(rng.choice([0, 3, 16, 128]))
        R = int(rng.choice([0, 2, 5, 16, 128]))
        B = int(rng.integers(1, 4))
        lens = [int(rng.integers(1, 1500)) for _ in range(B)]
        if i % 7 == 0:
            lens[0] = int(rng.choice([1, 14, 15, 16, 22, 23, (C - 1) * 8 + 15, (C - 1) * 8 + 16]))
        offs = [int(rng.integers(0, 50)) if i % 3 else 0 for _ in range(B)]
        xs = feats(lens, i)
        with torch.no_grad():
            r = enc.forward_parallel_chunk(xs, torch.tensor(lens), C, L, R,
                                           offset=torch.tensor(offs, dtype=torch.long))
        cases.append((C, L, R, B))
        out[f"c{i}_lens"] = np.array(lens, np.int32)
        out[f"c{i}_offs"] = np.array(offs, np.int32)
        out[f"c{i}_clr"] = np.array([C, L, R], np.int32)
        out[f"c{i}_att"] = np.packbits(cap["att"][:, 0].numpy().astype(bool), axis=-1)
        out[f"c{i}_att_shape"] = np.array(cap["att"][:, 0].shape, np.int32)
        out[f"c{i}_pad"] = np.packbits(cap["pad"][:, 0].numpy().astype(bool), axis=-1)
        out[f"c{i}_pad_shape"] = np.array(cap["pad"][:, 0].shape, np.int32)
        out[f"c{i}_nchunks"] = np.array(r[2], np.int32)
        out[f"c{i}_outlens"] = r[1].numpy().astype(np.int32)
        out[f"c{i}_offset_out"] = r[5].numpy().astype(np.int64)
    out["n_cases"] = np.array(len(cases))
    np.savez_compressed(path, **out)


# ---------------------------------------------------------------------------- small model
def endless_reference(enc, ctc, x, C, L, R, tbd):
    """Segment loop of ChunkFormerModel.endless_decode (chunkformer_model.py:344-438),
    driven on precomputed fbank (audio loading is unavailable offline)."""
    nb, d, H = enc.num_blocks, enc._output_size, enc.attention_heads
    sub, lorder = enc.embed.subsampling_rate, enc.cnn_module_kernel // 2
    max_len = int(tbd // 0.01) // 2
    mult = max_len // C // sub
    trunc = C * mult
    rel_right = (max(R, lorder) + max(C, max(R, lorder)) * (nb - 1)) * sub
    xs_len = x.shape[0]
    offset = torch.zeros(1, dtype=torch.int)
    att_cache = torch.zeros(nb, L, H, d * 2 // H)
    cnn_cache = torch.zeros(nb, d, lorder)
    outs = []
    for idx, _ in enumerate(range(0, xs_len, trunc * sub)):
        start = max(trunc * sub * idx, 0)
        end = min(trunc * sub * (idx + 1) + 7, xs_len)
        seg = x[start: end + rel_right]
        seg_len = torch.tensor([seg.shape[0]], dtype=torch.int)
        eo, el, _, att_cache, cnn_cache, offset = enc.forward_parallel_chunk(
            xs=[seg], xs_origin_lens=seg_len, chunk_size=C, left_context_size=L,
            right_context_size=R, att_cache=att_cache, cnn_cache=cnn_cache,
            truncated_context_size=trunc, offset=offset)
        eo = eo.reshape(1, -1, eo.shape[-1])[:, :el]
        if C * mult * sub * idx + rel_right < xs_len:
            eo = eo[:, :trunc]
        offset = offset - el + eo.shape[1]
        outs.append(eo)
        if C * mult * sub * idx + rel_right >= xs_len:
            break
    enc_out = torch.cat(outs, 1)
    ids = torch.argmax(ctc.log_softmax(enc_out).squeeze(0), dim=-1)
    return enc_out[0], ids, att_cache, cnn_cache, len(outs)


def gen_small(path, cfg=SMALL, seed=1):
    enc, ctc, sd = build_reference(cfg, seed)
    out = {"sd_digest": sd_digest(sd), "seed": np.array(seed)}
    cases = {
        "a": ([700, 237, 1100, 40, 14, 519, 135, 136], 16, 32, 32),
        "b": ([300, 77, 1], 8, 16, 4),
        "c": ([1234, 3000], 64, 128, 128),
        "d": ([500], 16, 0, 0),
    }
    with torch.no_grad():
        for name, (lens, C, L, R) in cases.items():
            xs = feats(lens, 100 + ord(name))
            r = enc.forward_parallel_chunk(xs, torch.tensor(lens), C, L, R)
            out[f"{name}_lens"] = np.array(lens, np.int32)
            out[f"{name}_clr"] = np.array([C, L, R], np.int32)
            out[f"{name}_seed"] = np.array(100 + ord(name))
            out[f"{name}_out"] = r[0].numpy()
            out[f"{name}_outlens"] = r[1].numpy()
            out[f"{name}_nchunks"] = np.array(r[2], np.int32)
            if name == "a":
                out["a_logp"] = ctc.log_softmax(r[0]).numpy()
        # cache path: batch of one with explicit caches and truncation
        xs = feats([900], 7)
        ac = torch.randn(cfg.num_blocks, 32, cfg.n_heads, 2 * cfg.head_dim, generator=torch.Generator().manual_seed(8)) * 0.5
        cc = torch.randn(cfg.num_blocks, cfg.d_model, 7, generator=torch.Generator().manual_seed(9)) * 0.5
        r = enc.forward_parallel_chunk(xs, torch.tensor([900]), 16, 32, 32, att_cache=ac.clone(),
                                       cnn_cache=cc.clone(), truncated_context_size=48,
                                       offset=torch.tensor([5], dtype=torch.int))
        out.update(cache_seed=np.array(7), cache_att_in=ac.numpy(), cache_cnn_in=cc.numpy(),
                   cache_out=r[0].numpy(), cache_att_out=r[3].numpy(), cache_cnn_out=r[4].numpy(),
                   cache_offset_out=r[5].numpy())
        # endless decode on a long utterance
        x = feats([6000], 11)[0]
        eo, ids, ac2, cc2, nseg = endless_reference(enc, ctc, x, 16, 32, 32, tbd=20)
        out.update(endless_seed=np.array(11), endless_out=eo.numpy(), endless_ids=ids.numpy(),
                   endless_att=ac2.numpy(), endless_cnn=cc2.numpy(), endless_nseg=np.array(nseg),
                   endless_clrt=np.array([16, 32, 32, 20], np.int32))
        # padded path (encode()): chunked and full attention
        lens = [300, 123, 17]
        xs = feats(lens, 21)
        T = max(lens)
        xp = torch.zeros(len(lens), T, 80)
        for i, t in enumerate(xs):
            xp[i, : t.shape[0]] = t
        for name, (C, L, R) in {"pc": (16, 32, 32), "pf": (0, 0, 0)}.items():
            y, masks = enc.forward_encoder(xp, torch.tensor(lens), C, L, R)
            out[f"{name}_seed"] = np.array(21)
            out[f"{name}_lens"] = np.array(lens, np.int32)
            out[f"{name}_clr"] = np.array([C, L, R], np.int32)
            out[f"{name}_out"] = y.numpy()
            out[f"{name}_mask"] = masks.numpy()
    np.savez_compressed(path, **out)


def gen_large(path, seed=0):
    cfg = LARGE
    enc, ctc, sd = build_reference(cfg, seed)
    lens = [1234, 600]
    xs = feats(lens, 5)
    with torch.no_grad():
        r = enc.forward_parallel_chunk(xs, torch.tensor(lens), 64, 128, 128)
        logp = ctc.log_softmax(r[0])
    top2 = torch.topk(logp, 2, dim=-1).values
    np.savez_compressed(path, sd_digest=sd_digest(sd), seed=np.array(seed), lens=np.array(lens, np.int32),
                        feat_seed=np.array(5), out=r[0].numpy(), outlens=r[1].numpy(),
                        nchunks=np.array(r[2], np.int32), ids=logp.argmax(-1).numpy().astype(np.int32),
                        top2=top2.numpy(), lse_row0=logp[0, 0].numpy())


if __name__ == "__main__":
    which = sys.argv[1:] or ["masks", "small", "large"]
    if "masks" in which:
        gen_masks(os.path.join(HERE, "masks.npz"))
    if "small" in which:
        gen_small(os.path.join(HERE, "small.npz"))
    if "large" in which:
        gen_large(os.path.join(HERE, "large.npz"))
    print("ok", which)
