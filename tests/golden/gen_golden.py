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

from chunkformer_amd.config import LARGE, LARGE_4H, SMALL, SMALL256, EncoderConfig  # noqa: E402
from chunkformer_amd.weights import synthetic_features, synthetic_state_dict, synthetic_vocab  # noqa: E402

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
    """chunkformer-large, 12 layers: a 30 s utterance (configs[0]'s shape, 3000 frames) next to two
    shorter ones in one masked batch (C=64, L=R=128), plus CTC ids and top-2 margins."""
    cfg = LARGE
    enc, ctc, sd = build_reference(cfg, seed)
    lens = [3000, 1234, 600]
    xs = feats(lens, 5)
    with torch.no_grad():
        r = enc.forward_parallel_chunk(xs, torch.tensor(lens), 64, 128, 128)
        logp = ctc.log_softmax(r[0])
    top2 = torch.topk(logp, 2, dim=-1).values
    np.savez_compressed(path, sd_digest=sd_digest(sd), seed=np.array(seed), lens=np.array(lens, np.int32),
                        feat_seed=np.array(5), out=r[0].numpy(), outlens=r[1].numpy(),
                        nchunks=np.array(r[2], np.int32), ids=logp.argmax(-1).numpy().astype(np.int32),
                        top2=top2.numpy(), lse_row0=logp[0, 0].numpy())


def gen_large_4h(path, seed=0):
    """d=512 with 4 heads (head_dim 128), the family of the reference's large vie recipe."""
    cfg = LARGE_4H
    enc, ctc, sd = build_reference(cfg, seed)
    lens = [1234, 600]
    xs = feats(lens, 6)
    with torch.no_grad():
        r = enc.forward_parallel_chunk(xs, torch.tensor(lens), 64, 128, 128)
        logp = ctc.log_softmax(r[0])
        # padded chunked path (encode()) on the same utterances
        xp = torch.zeros(len(lens), max(lens), 80)
        for i, t in enumerate(xs):
            xp[i, : t.shape[0]] = t
        y, masks = enc.forward_encoder(xp, torch.tensor(lens), 64, 128, 128)
    top2 = torch.topk(logp, 2, dim=-1).values
    np.savez_compressed(path, sd_digest=sd_digest(sd), seed=np.array(seed), lens=np.array(lens, np.int32),
                        feat_seed=np.array(6), out=r[0].numpy(), outlens=r[1].numpy(),
                        nchunks=np.array(r[2], np.int32), ids=logp.argmax(-1).numpy().astype(np.int32),
                        top2=top2.numpy(), pc_out=y.numpy(), pc_mask=masks.numpy())


ENDLESS_LAYERS = [0, 6, 11]   # att_cache layers stored (the full [12,128,8,128] stack is 6 MB)


def gen_large_endless(path, seed=0):
    """configs[3] geometry on chunkformer-large: C=64, L=R=128, 12 layers, tbd=20 -> 4 segments of
    <= 12,807 frames with the att/cnn caches and offset carried; final caches recorded."""
    cfg = LARGE
    enc, ctc, sd = build_reference(cfg, seed)
    x = feats([13500], 12)[0]
    with torch.no_grad():
        eo, ids, ac, cc, nseg = endless_reference(enc, ctc, x, 64, 128, 128, tbd=20)
    assert nseg >= 3, nseg
    np.savez_compressed(path, sd_digest=sd_digest(sd), seed=np.array(seed), feat_seed=np.array(12),
                        T=np.array(13500), clrt=np.array([64, 128, 128, 20], np.int32), nseg=np.array(nseg),
                        out=eo.numpy(), ids=ids.numpy().astype(np.int32),
                        att_layers=np.array(ENDLESS_LAYERS, np.int32),
                        att=ac[ENDLESS_LAYERS].numpy(), cnn=cc.numpy())


def gen_large_full(path, seed=0):
    """configs[4] geometry on chunkformer-large: full attention (chunk_size 0 -> T'), padded batch of a
    30 s utterance and a 21 s one (key padding mask), 12 layers."""
    cfg = LARGE
    enc, _, sd = build_reference(cfg, seed)
    lens = [3000, 2100]
    xs = feats(lens, 13)
    xp = torch.zeros(len(lens), max(lens), 80)
    for i, t in enumerate(xs):
        xp[i, : t.shape[0]] = t
    with torch.no_grad():
        y, masks = enc.forward_encoder(xp, torch.tensor(lens), 0, 0, 0)
    np.savez_compressed(path, sd_digest=sd_digest(sd), seed=np.array(seed), feat_seed=np.array(13),
                        lens=np.array(lens, np.int32), out=y.numpy(), mask=masks.numpy())


FULL_MIXED_LENS = [3000, 2987, 2456, 1900, 1333, 1001, 640, 333, 96]


def gen_large_full_mixed(path, seed=0):
    """configs[4] as the bench runs it, at 9 utterances: full attention (chunk_size 0) over a padded batch
    of mixed lengths (30 s down to 1 s: every key-padding case of the dense kernel, T' = 374 .. 11), 12
    layers, with the CTC head's ids and top-2 margins; only the valid rows are stored."""
    cfg = LARGE
    enc, ctc, sd = build_reference(cfg, seed)
    lens = FULL_MIXED_LENS
    xs = feats(lens, 17)
    xp = torch.zeros(len(lens), max(lens), 80)
    for i, t in enumerate(xs):
        xp[i, : t.shape[0]] = t
    with torch.no_grad():
        y, masks = enc.forward_encoder(xp, torch.tensor(lens), 0, 0, 0)
        logp = ctc.log_softmax(y)
    valid = masks[:, 0, :].numpy()
    top2 = torch.topk(logp, 2, dim=-1).values.numpy()[valid]
    np.savez_compressed(path, sd_digest=sd_digest(sd), seed=np.array(seed), feat_seed=np.array(17),
                        lens=np.array(lens, np.int32), mask=masks.numpy(), out=y.numpy()[valid],
                        ids=logp.argmax(-1).numpy()[valid].astype(np.int32), margin=top2[:, 0] - top2[:, 1])


def gen_text(path):
    """Text post-processing of the reference (utils/model_utils.py: get_output 164-171,
    get_output_with_timestamps 174-221) on (a) seeded id streams with long blank runs and repeats,
    (b) the CTC ids of large_4h.npz per utterance (the checkpoint-loader test decodes them);
    vocabulary: chunkformer_amd.weights.synthetic_vocab.  model_utils imports torchaudio.functional
    at module level (unused by these functions): an empty stub module stands in for it."""
    import json
    ta = types.ModuleType("torchaudio")
    taf = types.ModuleType("torchaudio.functional")
    ta.functional = taf
    sys.modules.setdefault("torchaudio", ta)
    sys.modules.setdefault("torchaudio.functional", taf)
    from chunkformer.utils import model_utils as mu
    V = 5000
    cd = synthetic_vocab(V)
    rng = np.random.default_rng(7)
    streams = []
    for n in (1, 7, 40, 150, 400, 999):
        ids, t = [], 0
        while len(ids) < n:
            if rng.random() < 0.55:
                ids += [0] * int(rng.integers(1, 14))
            else:
                ids += [int(rng.integers(1, V))] * int(rng.integers(1, 4))
        streams.append(ids[:n])
    out = {"V": V, "streams": streams,
           "get_output": mu.get_output(streams, cd, "asr_model"),
           "timestamps": {str(ms): mu.get_output_with_timestamps([torch.tensor(s).reshape(-1, 1) for s in streams],
                                                                 cd, "asr_model", ms)
                          for ms in (0.5, 0.24, 1.0)}}
    # transducer branch (model_type "transducer"): per-frame decision rows [T, n_steps], no collapse
    tstreams = []
    for T in (1, 9, 60, 333):
        d = np.zeros((T, 4), np.int64)
        for t in range(T):
            if rng.random() < 0.4:
                k = int(rng.integers(1, 4))
                d[t, :k] = rng.integers(1, V, size=k)
        tstreams.append(d)
    out["transducer_streams"] = [d.tolist() for d in tstreams]
    out["transducer_timestamps"] = {str(ms): mu.get_output_with_timestamps([torch.tensor(d) for d in tstreams], cd,
                                                                           "transducer", ms)
                                    for ms in (0.5, 0.24, 0.0, 1.0)}
    g = np.load(os.path.join(HERE, "large_4h.npz"))
    starts = np.cumsum([0] + g["nchunks"].tolist())
    hyps = [g["ids"][starts[u]: starts[u + 1]].reshape(-1)[: int(n)].tolist() for u, n in enumerate(g["outlens"])]
    out["large_4h_decode"] = mu.get_output(hyps, cd, "asr_model")
    with open(path, "w", encoding="utf8") as f:
        json.dump(out, f, ensure_ascii=False)


STREAM_LAYERS = [0, 11]   # att_cache layers stored for the 12-layer run


def stream_reference(enc, xs_steps, C, L, R, B):
    """The realtime loop (apps/realtime-asr/stream_asr.py:105-180): zero caches [nb, B, H, L, 2dk] /
    [nb, B, d, 7], encoder.forward_chunk per step with the caches carried and offset += C."""
    nb, d, H = enc.num_blocks, enc._output_size, enc.attention_heads
    att = torch.zeros(nb, B, H, L, 2 * d // H)
    cnn = torch.zeros(nb, B, d, enc.cnn_module_kernel // 2)
    offset, outs = 0, []
    for x in xs_steps:
        y, _, att, cnn = enc.forward_chunk(x, att_cache=att, cnn_cache=cnn, chunk_size=C, left_context_size=L,
                                           right_context_size=R, offset=offset)
        outs.append(y)
        offset += C
    return outs, att, cnn


def gen_stream(path):
    """forward_chunk (encoder.py:310-385) streaming steps: (a) the small model, batch of 2, C=16
    L=32 R=16: four full steps (T' = C + R) and a short last step (T' = 27); (b) the 4-head d=512
    12-layer model (head_dim 128), C=64 L=R=128, three full steps (T' = 192)."""
    out = {}
    with torch.no_grad():
        enc, _, sd = build_reference(SMALL, 1)
        C, L, R = 16, 32, 16
        Tps = [C + R] * 4 + [27]
        steps = [torch.stack(feats([8 * (tp - 1) + 15] * 2, 300 + i)) for i, tp in enumerate(Tps)]
        outs, att, cnn = stream_reference(enc, steps, C, L, R, 2)
        out.update(a_clr=np.array([C, L, R], np.int32), a_tp=np.array(Tps, np.int32), a_B=np.array(2),
                   a_seed0=np.array(300), a_att=att.numpy(), a_cnn=cnn.numpy())
        for i, y in enumerate(outs):
            out[f"a_out{i}"] = y.numpy()
        enc, _, sd = build_reference(LARGE_4H, 0)
        C, L, R = 64, 128, 128
        Tps = [C + R] * 3
        steps = [torch.stack(feats([8 * (tp - 1) + 15], 400 + i)) for i, tp in enumerate(Tps)]
        outs, att, cnn = stream_reference(enc, steps, C, L, R, 1)
        out.update(b_clr=np.array([C, L, R], np.int32), b_tp=np.array(Tps, np.int32), b_B=np.array(1),
                   b_seed0=np.array(400), b_att_layers=np.array(STREAM_LAYERS, np.int32),
                   b_att=att[STREAM_LAYERS].numpy(), b_cnn=cnn.numpy())
        for i, y in enumerate(outs):
            out[f"b_out{i}"] = y.numpy()
    np.savez_compressed(path, **out)


def gen_chunk_by_chunk(path, cfg=SMALL, seed=1):
    """forward_chunk_by_chunk (encoder.py:387-459): the reference's own streaming loop over forward_chunk
    (input padded to the stride, caches carried, every chunk's first chunk_size rows kept but the last
    one's whole output), batch of 2 utterances of different lengths, two geometries."""
    enc, _, sd = build_reference(cfg, seed)
    out = {"sd_digest": sd_digest(sd), "seed": np.array(seed)}
    cases = [("a", [1003, 777], 16, 32, 16, 61), ("b", [640, 640], 8, 16, 8, 62)]
    with torch.no_grad():
        for tag, lens, C, L, R, fs in cases:
            xs = feats(lens, fs)
            xp = torch.zeros(len(lens), max(lens), 80)
            for i, t in enumerate(xs):
                xp[i, : t.shape[0]] = t
            y, masks = enc.forward_chunk_by_chunk(xp, torch.tensor(lens), C, L, R)
            out.update({f"{tag}_lens": np.array(lens, np.int32), f"{tag}_clr": np.array([C, L, R], np.int32),
                        f"{tag}_feat_seed": np.array(fs), f"{tag}_out": y.numpy(), f"{tag}_mask": masks.numpy()})
    np.savez_compressed(path, **out)


def gen_endless_tbd(path, cfg=SMALL, seed=1):
    """The small endless input of small.npz decoded again with total_batch_duration 80 (2 segments
    instead of 7): the reference's output depends (slightly) on the segmentation, so the bench's
    larger segments are pinned at their own tbd."""
    enc, ctc, sd = build_reference(cfg, seed)
    x = feats([6000], 11)[0]
    with torch.no_grad():
        eo, ids, ac, cc, nseg = endless_reference(enc, ctc, x, 16, 32, 32, tbd=80)
    np.savez_compressed(path, sd_digest=sd_digest(sd), seed=np.array(seed), feat_seed=np.array(11),
                        clrt=np.array([16, 32, 32, 80], np.int32), nseg=np.array(nseg), out=eo.numpy(),
                        ids=ids.numpy().astype(np.int32), att=ac.numpy(), cnn=cc.numpy())


def gen_tiny_padded(path, cfg=SMALL, seed=1):
    """The padded path (forward_encoder, chunked and full attention) on a batch with 5- and 3-frame
    utterances (calc_length -1: a mask with no valid frame, every attention row of theirs fully masked)."""
    enc, ctc, sd = build_reference(cfg, seed)
    lens = [300, 5, 17, 3]
    xs = feats(lens, 23)
    xp = torch.zeros(len(lens), max(lens), 80)
    for i, t in enumerate(xs):
        xp[i, : t.shape[0]] = t
    out = {"sd_digest": sd_digest(sd), "seed": np.array(seed), "feat_seed": np.array(23),
           "lens": np.array(lens, np.int32)}
    with torch.no_grad():
        for name, (C, L, R) in {"pc": (16, 32, 32), "pf": (0, 0, 0)}.items():
            y, masks = enc.forward_encoder(xp, torch.tensor(lens), C, L, R)
            out[f"{name}_clr"] = np.array([C, L, R], np.int32)
            out[f"{name}_out"] = y.numpy()
            out[f"{name}_mask"] = masks.numpy()
            print(name, tuple(y.shape), masks.squeeze(1).sum(-1).tolist(), bool(torch.isfinite(y).all()))
    np.savez_compressed(path, **out)


TINY_BATCH_LENS = (5, 300, 3, 14, 15, 700, 6, 7)


def gen_tiny_batch(path, cfg=SMALL, seed=1):
    """batch_decode's asr branch (chunkformer_model.py:524-531) on a batch with utterances of 3-15
    frames: calc_length -1 (< 7 frames) makes hyp.flatten()[:x_len] keep all but the last id of the
    padded chunk, 0 keeps none; the ids and the get_output strings (model_utils.py:164-171, vocabulary
    synthetic_vocab) of every utterance."""
    ta = types.ModuleType("torchaudio")
    taf = types.ModuleType("torchaudio.functional")
    ta.functional = taf
    sys.modules.setdefault("torchaudio", ta)
    sys.modules.setdefault("torchaudio.functional", taf)
    from chunkformer.utils import model_utils as mu
    enc, ctc, sd = build_reference(cfg, seed)
    lens = list(TINY_BATCH_LENS)
    xs = feats(lens, 29)
    with torch.no_grad():
        eo, el, n_chunks, _, _, _ = enc.forward_parallel_chunk(
            xs=xs, xs_origin_lens=torch.tensor(lens, dtype=torch.int), chunk_size=16, left_context_size=32,
            right_context_size=32, offset=torch.zeros(len(lens), dtype=torch.int))
        logp = ctc.log_softmax(eo)
        hyps = torch.argmax(logp, dim=-1).split(n_chunks, dim=0)
        hyps = [h.flatten()[:n] for h, n in zip(hyps, el)]
        top2 = logp.topk(2, dim=-1).values
        margin = (top2[..., 0] - top2[..., 1]).split(n_chunks, dim=0)
        margin = [m.flatten()[:n] for m, n in zip(margin, el)]
    texts = mu.get_output(hyps, synthetic_vocab(cfg.vocab), "asr_model")
    np.savez_compressed(path, sd_digest=sd_digest(sd), seed=np.array(seed), feat_seed=np.array(29),
                        clr=np.array([16, 32, 32], np.int32), lens=np.array(lens, np.int32),
                        outlens=el.numpy().astype(np.int32), nchunks=np.array(n_chunks, np.int32),
                        hyp_lens=np.array([h.numel() for h in hyps], np.int32),
                        hyps=torch.cat(hyps).numpy().astype(np.int32), margins=torch.cat(margin).numpy(),
                        texts=np.array(texts))
    print("tiny batch:", el.tolist(), [h.numel() for h in hyps], texts)


ENDLESS_TAIL_LENS = (897, 900, 910, 911, 918, 1796)


def gen_endless_tail(path, cfg=SMALL, seed=1):
    """endless_decode (tbd 20, C 16, L = R = 32: 896-frame steps) on inputs whose LAST segment is
    1-22 frames: calc_length of a segment under 15 frames is <= 0 (-1 below 7 frames), and the
    reference's encoder_out[:, :encoder_len] (chunkformer_model.py:419) then keeps all but the
    last row of the segment's padded chunk (-1) or nothing (0).  Pins that slicing for every
    endless mode (a graph-replayed ragged last segment took -1 as a row count)."""
    enc, ctc, sd = build_reference(cfg, seed)
    out = {"sd_digest": sd_digest(sd), "seed": np.array(seed), "feat_seed": np.array(13),
           "clrt": np.array([16, 32, 32, 20], np.int32), "lens": np.array(ENDLESS_TAIL_LENS, np.int32)}
    with torch.no_grad():
        for n in ENDLESS_TAIL_LENS:
            x = feats([n], 13)[0]
            eo, ids, ac, cc, nseg = endless_reference(enc, ctc, x, 16, 32, 32, tbd=20)
            out.update({f"out_{n}": eo.numpy(), f"ids_{n}": ids.numpy().astype(np.int32), f"att_{n}": ac.numpy(),
                        f"cnn_{n}": cc.numpy(), f"nseg_{n}": np.array(nseg)})
            print(f"endless tail {n}: {nseg} segments, {eo.shape[0]} rows")
    np.savez_compressed(path, **out)


PEAK_SECTORS, PEAK_BLANK, PEAK_SCALE, PEAK_REST = 16, 0.8, 2.0, 0.1


def peaked_ctc_head(out, sd, sectors=PEAK_SECTORS, blank=PEAK_BLANK, scale=PEAK_SCALE, rest=PEAK_REST):
    """A peaked ctc_lo for a random-weight encoder, standing in for a trained head.

    Scaling the seeded head does not make it peaked in the sense that matters: its argmax margins
    and the logit error of a bf16 encoder grow together (the seeded encoder's frames share one
    dominant direction, |x - mean| / |x| ~ 0.3, and the top-2 rows of a random V=1024 head nearly
    tie).  A trained head reads the directions the frames vary along, so this one does: token rows
    are `sectors` unit directions in the whitened plane of the reference outputs' two leading
    principal components (centred on their mean, which the bias removes), the blank row wins
    inside radius `blank`, and every other row is the seeded row x `rest` with bias -8.  All the
    logits are scaled by `scale`.  Returns (rows, w_rows, bias) for with_fixture_ctc_head."""
    x = out.reshape(-1, out.shape[-1]).double()
    mu = x.mean(0)
    _, s, vh = torch.linalg.svd(x - mu, full_matrices=False)
    sig = s / x.shape[0] ** 0.5
    th = torch.arange(sectors, dtype=torch.float64) * (2 * np.pi / sectors)
    d = torch.cos(th)[:, None] * vh[0] / sig[0] + torch.sin(th)[:, None] * vh[1] / sig[1]
    V = sd["ctc.ctc_lo.weight"].shape[0]
    rows = torch.cat([torch.tensor([0]), 1 + torch.arange(sectors) * ((V - 1) // sectors)])
    w_rows = torch.cat([torch.zeros(1, x.shape[1], dtype=torch.float64), scale * d]).float()
    bias = torch.full((V,), -8.0)
    bias[rows[1:]] = (-(scale * d) @ mu).float()
    bias[0] = scale * blank
    return rows.numpy().astype(np.int32), w_rows.numpy(), bias.numpy()


def gen_small256(path, seed=2):
    """The reference's shipped small recipes (examples/asr/ctc/conf/chunkformer-ctc-small-libri-100h.yaml:5-8,
    likewise the rnnt-small and libri-960h recipes): d=256, 4 heads (head_dim 64), ff 2048, 12 blocks,
    bpe1024 vocabulary.  (a) masked batch at the decoding default C=64 L=R=128 with CTC ids and top-2
    margins under a peaked head (peaked_ctc_head; reference median top-2 margin >= 0.5); (b) the
    padded chunked path (encode()) on the same utterances; (c) a masked batch with C=128 L=R=128
    (one of the recipe's dynamic_chunk_sizes, > 64 queries per chunk)."""
    cfg = SMALL256
    enc, ctc, sd = build_reference(cfg, seed)
    lens = [3000, 1234, 600]
    xs = feats(lens, 8)
    with torch.no_grad():
        r = enc.forward_parallel_chunk(xs, torch.tensor(lens), 64, 128, 128)
        rows, w_rows, bias = peaked_ctc_head(r[0], sd)
        w = sd["ctc.ctc_lo.weight"] * PEAK_REST
        w[torch.from_numpy(rows.astype(np.int64))] = torch.from_numpy(w_rows)
        ctc.ctc_lo.weight.data.copy_(w)
        ctc.ctc_lo.bias.data.copy_(torch.from_numpy(bias))
        logp = ctc.log_softmax(r[0])
        xp = torch.zeros(len(lens), max(lens), 80)
        for i, t in enumerate(xs):
            xp[i, : t.shape[0]] = t
        y, masks = enc.forward_encoder(xp, torch.tensor(lens), 64, 128, 128)
        r2 = enc.forward_parallel_chunk(xs, torch.tensor(lens), 128, 128, 128)
    top2 = torch.topk(logp, 2, dim=-1).values
    mg = (top2[..., 0] - top2[..., 1]).flatten()
    ids = logp.argmax(-1).flatten()
    print(f"small256 peaked head: median top-2 margin {float(mg.median()):.3f}, min {float(mg.min()):.2e}, "
          f"blank {float((ids == 0).float().mean()):.2f}, ids used {int(ids.unique().numel())}")
    np.savez_compressed(path, sd_digest=sd_digest(sd), seed=np.array(seed), lens=np.array(lens, np.int32),
                        ctc_rows=rows, ctc_w_rows=w_rows, ctc_bias=bias, ctc_rest_scale=np.array(PEAK_REST),
                        feat_seed=np.array(8), out=r[0].numpy(), outlens=r[1].numpy(),
                        nchunks=np.array(r[2], np.int32), ids=logp.argmax(-1).numpy().astype(np.int32),
                        top2=top2.numpy(), pc_out=y.numpy(), pc_mask=masks.numpy(),
                        c128_out=r2[0].numpy(), c128_nchunks=np.array(r2[2], np.int32), c128_outlens=r2[1].numpy())


def gen_rows_neq(path, cfg=SMALL, seed=1):
    """forward_parallel_chunk with x.size(0) != xs_origin_lens (encoder.py:556-596, 673): the rows are
    padded and unfolded from x.size(0) while the masks and output lengths follow xs_origin_lens; the
    lengths keep the reference's bound count equal to its window count (else it fails on shapes)."""
    enc, _, sd = build_reference(cfg, seed)
    rows, lens, C, L, R = [700, 237, 1100, 300], [690, 230, 1100, 271], 16, 32, 32
    xs = feats(rows, 55)
    # (gt) the other direction, xs_origin_lens > x.size(0) with equal chunk counts (690 rows, lens 695;
    # 240 rows, lens 245): the masks reach past the real rows, which the reference fills with zeros
    gt_rows, gt_lens = [690, 240, 500], [695, 245, 500]
    gt_xs = feats(gt_rows, 56)
    with torch.no_grad():
        r = enc.forward_parallel_chunk(xs, torch.tensor(lens), C, L, R)
        r2 = enc.forward_parallel_chunk(gt_xs, torch.tensor(gt_lens), C, L, R)
    np.savez_compressed(path, sd_digest=sd_digest(sd), seed=np.array(seed), feat_seed=np.array(55),
                        rows=np.array(rows, np.int32), lens=np.array(lens, np.int32), clr=np.array([C, L, R], np.int32),
                        out=r[0].numpy(), outlens=r[1].numpy(), nchunks=np.array(r[2], np.int32),
                        gt_feat_seed=np.array(56), gt_rows=np.array(gt_rows, np.int32),
                        gt_lens=np.array(gt_lens, np.int32), gt_out=r2[0].numpy(), gt_outlens=r2[1].numpy(),
                        gt_nchunks=np.array(r2[2], np.int32))


ENDLESS_RNNT_FRAMES = 480


def gen_rnnt(path, seed=3, n_steps=64):
    """The RNN-T consumer (chunkformer_model.py:439-448, 533-543): the reference's optimized_search /
    batch_greedy_search (transducer/search/greedy_search.py:6-92) with its RNNPredictor (lstm) and
    TransducerJoint built from the vie recipe's shapes (examples/asr/rnnt/conf/
    chunkformer-rnnt-large-vie.yaml: embed 256, hidden 512 x 2 layers, output 512, join 512,
    V = 1024) and seeded weights (chunkformer_amd.transducer.synthetic_transducer_state_dict), over
    encoder outputs the reference produced: (a) large_4h.npz's two utterances as one padded batch
    (batch_decode's call) and (b) the first ENDLESS_RNNT_FRAMES frames of large_endless.npz's
    4-segment output (endless_decode's call, B=1)."""
    from chunkformer.transducer.joint import TransducerJoint
    from chunkformer.transducer.predictor import RNNPredictor
    from chunkformer.transducer.search.greedy_search import batch_greedy_search, optimized_search

    from chunkformer_amd.transducer import RNNTConfig, synthetic_transducer_state_dict
    c = RNNTConfig()
    sd = synthetic_transducer_state_dict(c, seed)
    pred = RNNPredictor(c.vocab, c.embed_size, c.pred_out, 0.1, c.hidden, c.num_layers, True, "lstm", 0.1).eval()
    joint = TransducerJoint(c.vocab, c.enc_dim, c.pred_out, c.join_dim, True, False, "add", "tanh").eval()
    pred.load_state_dict({k[len("predictor."):]: v for k, v in sd.items() if k.startswith("predictor.")}, strict=True)
    joint.load_state_dict({k[len("joint."):]: v for k, v in sd.items() if k.startswith("joint.")}, strict=True)
    model = types.SimpleNamespace(predictor=pred, joint=joint, blank=0)
    g4 = np.load(os.path.join(HERE, "large_4h.npz"))
    starts = np.cumsum([0] + g4["nchunks"].tolist())
    utts = [torch.from_numpy(g4["out"][starts[u]: starts[u + 1]].reshape(-1, c.enc_dim)[: int(n)])
            for u, n in enumerate(g4["outlens"])]
    lens = torch.tensor([u.shape[0] for u in utts])
    enc_b = torch.nn.utils.rnn.pad_sequence(utts, batch_first=True)
    ge = np.load(os.path.join(HERE, "large_endless.npz"))
    enc_e = torch.from_numpy(ge["out"][:ENDLESS_RNNT_FRAMES]).unsqueeze(0)
    with torch.no_grad():
        out_b = optimized_search(model, enc_b, lens, n_steps)
        hyps_b = batch_greedy_search(model, enc_b, lens, n_steps)
        out_e = optimized_search(model, enc_e, torch.tensor([enc_e.shape[1]]), n_steps)
    from oracle import rnnt_ref
    _, m_b = rnnt_ref.optimized_search(sd, c.num_layers, c.hidden, enc_b, lens, n_steps)
    _, m_e = rnnt_ref.optimized_search(sd, c.num_layers, c.hidden, enc_e, [enc_e.shape[1]], n_steps)
    for nm, o in (("batch", out_b), ("endless", out_e)):
        d = o.reshape(o.shape[0], -1, n_steps)
        first = d[..., 0]
        print(f"rnnt {nm}: frames {first.numel()}, blank-first {float((first == 0).float().mean()):.3f}, "
              f"tokens {int((d != 0).sum())}, max steps/frame {int((d != 0).sum(-1).max())}")
    print(f"rnnt min top-2 margins: batch {m_b:.2e}, endless {m_e:.2e}")
    flat = [t for h in hyps_b for t in h]
    np.savez_compressed(path, seed=np.array(seed), n_steps=np.array(n_steps),
                        vocab=np.array(c.vocab), batch_lens=lens.numpy().astype(np.int32),
                        batch_out=out_b.numpy().astype(np.int32), batch_hyp_lens=np.array([len(h) for h in hyps_b]),
                        batch_hyps=np.array(flat, np.int32), endless_out=out_e.numpy().astype(np.int32),
                        margin_batch=np.array(m_b), margin_endless=np.array(m_e))


SPARSE_BLANK_BIAS = 7.0   # with enc_scale 8: 80% of the frames decide blank first
SPARSE_ENC_SCALE = 8.0


def gen_rnnt_sparse(path, seed=3, n_steps=64, blank_bias=SPARSE_BLANK_BIAS, enc_scale=SPARSE_ENC_SCALE):
    """As gen_rnnt's endless half (optimized_search, B=1, the first ENDLESS_RNNT_FRAMES rows of
    large_endless.npz) with a larger blank bias and a frame-dependent joint (enc_ffn x8), so that
    blank dominates: 80% of the frames decide blank at their first step, in runs (the regime where
    the kernel's 8-frame blank-block skip decides most frames); decisions at n_steps 64 and 3."""
    from chunkformer.transducer.joint import TransducerJoint
    from chunkformer.transducer.predictor import RNNPredictor
    from chunkformer.transducer.search.greedy_search import optimized_search

    from chunkformer_amd.transducer import RNNTConfig, synthetic_transducer_state_dict
    c = RNNTConfig()
    sd = synthetic_transducer_state_dict(c, seed, blank_bias=blank_bias, enc_scale=enc_scale)
    pred = RNNPredictor(c.vocab, c.embed_size, c.pred_out, 0.1, c.hidden, c.num_layers, True, "lstm", 0.1).eval()
    joint = TransducerJoint(c.vocab, c.enc_dim, c.pred_out, c.join_dim, True, False, "add", "tanh").eval()
    pred.load_state_dict({k[len("predictor."):]: v for k, v in sd.items() if k.startswith("predictor.")}, strict=True)
    joint.load_state_dict({k[len("joint."):]: v for k, v in sd.items() if k.startswith("joint.")}, strict=True)
    model = types.SimpleNamespace(predictor=pred, joint=joint, blank=0)
    ge = np.load(os.path.join(HERE, "large_endless.npz"))
    enc_e = torch.from_numpy(ge["out"][:ENDLESS_RNNT_FRAMES]).unsqueeze(0)
    with torch.no_grad():
        out_e = optimized_search(model, enc_e, torch.tensor([enc_e.shape[1]]), n_steps)
        out_3 = optimized_search(model, enc_e, torch.tensor([enc_e.shape[1]]), 3)
    from oracle import rnnt_ref
    _, m_e = rnnt_ref.optimized_search(sd, c.num_layers, c.hidden, enc_e, [enc_e.shape[1]], n_steps)
    _, m_3 = rnnt_ref.optimized_search(sd, c.num_layers, c.hidden, enc_e, [enc_e.shape[1]], 3)
    m_e = min(m_e, m_3)
    d = out_e.reshape(1, -1, n_steps)
    first = d[..., 0]
    print(f"rnnt sparse: frames {first.numel()}, blank-first {float((first == 0).float().mean()):.3f}, "
          f"tokens {int((d != 0).sum())}, max steps/frame {int((d != 0).sum(-1).max())}, min margin {m_e:.2e}")
    np.savez_compressed(path, seed=np.array(seed), n_steps=np.array(n_steps), vocab=np.array(c.vocab),
                        blank_bias=np.array(blank_bias), enc_scale=np.array(enc_scale), endless_out=out_e.numpy().astype(np.int32),
                        endless_out_steps3=out_3.numpy().astype(np.int32),
                        margin_endless=np.array(m_e))


def gen_autocast(path, seed=0):
    """The reference decoder's --autocast_dtype fp16 / bf16 (chunkformer_model.py:709-743: the whole
    decode under torch.autocast): chunkformer-large masked batch at C=64 L=R=128 over four utterances,
    run in f32 and under CPU autocast float16 and bfloat16, with the CTC ids of each run.  Outputs are
    stored as float16 (after_norm outputs of magnitude < 64: a relative rounding of 2^-11, below
    the 1.4e-3 the fp16 run differs from f32 by)."""
    cfg = LARGE
    enc, ctc, sd = build_reference(cfg, seed)
    lens = [3000, 2500, 1234, 600]
    xs = feats(lens, 6)
    res = {}
    with torch.no_grad():
        r = enc.forward_parallel_chunk(xs, torch.tensor(lens), 64, 128, 128)
        ref = r[0].float()
        logp = ctc.log_softmax(ref)
        res["out_f32"] = ref.numpy().astype(np.float16)
        res["ids"] = logp.argmax(-1).numpy().astype(np.int32)
        top2 = torch.topk(logp, 2, dim=-1).values
        res["margin"] = (top2[..., 0] - top2[..., 1]).numpy()
        for name, dt in (("f16", torch.float16), ("bf16", torch.bfloat16)):
            with torch.autocast("cpu", dtype=dt):
                ra = enc.forward_parallel_chunk(xs, torch.tensor(lens), 64, 128, 128)
                la = ctc.log_softmax(ra[0])
            o = ra[0].float()
            rel = float((o - ref).norm() / ref.norm())
            ids = la.float().argmax(-1).numpy().astype(np.int32)
            print(f"autocast {name}: rel-L2 vs f32 {rel:.3e}, CTC ids equal {float((ids == res['ids']).mean()):.4f}")
            res[f"out_{name}"] = o.numpy().astype(np.float16)
            res[f"ids_{name}"] = ids
            res[f"rel_{name}"] = np.array(rel)
    np.savez_compressed(path, sd_digest=sd_digest(sd), seed=np.array(seed), lens=np.array(lens, np.int32),
                        feat_seed=np.array(6), nchunks=np.array(r[2], np.int32), outlens=r[1].numpy(), **res)


MEMORY_TOKENS, MEMORY_FORGET, MEMORY_SUPPRESS, MEMORY_THRESH = 64, 0.5, 100.0, 1.5


def gen_rnnt_memory(path, seed=3, n_steps=64, dir_seed=11):
    """The regime of a trained transducer: most non-blank frames emit 1-3 tokens and then stop on
    blank, below the n_steps cap.  Seeded weights reshaped by
    chunkformer_amd.transducer.with_emission_memory: MEMORY_TOKENS tokens, token k carried by the
    frames whose standardised projection on a seeded random direction w_k exceeds MEMORY_THRESH,
    and a decaying per-token memory in the predictor that turns a just-emitted token off.  The
    directions are standardised on the first ENDLESS_RNNT_FRAMES rows of large_endless.npz.
    optimized_search (transducer/search/greedy_search.py:6-74) over (a) those rows, B = 1, and (b)
    large_4h.npz's two utterances as one padded batch (+ batch_greedy_search's hypotheses)."""
    from chunkformer.transducer.joint import TransducerJoint
    from chunkformer.transducer.predictor import RNNPredictor
    from chunkformer.transducer.search.greedy_search import batch_greedy_search, optimized_search

    from chunkformer_amd.transducer import RNNTConfig, synthetic_transducer_state_dict, with_emission_memory
    c = RNNTConfig()
    ge = np.load(os.path.join(HERE, "large_endless.npz"))
    enc_e = torch.from_numpy(ge["out"][:ENDLESS_RNNT_FRAMES]).unsqueeze(0)
    x = enc_e[0].double()
    mu = x.mean(0)
    gen = torch.Generator().manual_seed(dir_seed)
    w = torch.randn(MEMORY_TOKENS, c.enc_dim, generator=gen, dtype=torch.float64)
    w /= w.norm(dim=1, keepdim=True)
    d = w / ((x - mu) @ w.T).std(0)[:, None]
    frame_dirs = d.float()
    frame_bias = (-(d @ mu) - MEMORY_THRESH).float()
    tokens = [1 + k * ((c.vocab - 1) // MEMORY_TOKENS) for k in range(MEMORY_TOKENS)]
    sd = with_emission_memory(synthetic_transducer_state_dict(c, seed), c, frame_dirs, frame_bias, tokens,
                              forget=MEMORY_FORGET, suppress=MEMORY_SUPPRESS)
    pred = RNNPredictor(c.vocab, c.embed_size, c.pred_out, 0.1, c.hidden, c.num_layers, True, "lstm", 0.1).eval()
    joint = TransducerJoint(c.vocab, c.enc_dim, c.pred_out, c.join_dim, True, False, "add", "tanh").eval()
    pred.load_state_dict({k[len("predictor."):]: v for k, v in sd.items() if k.startswith("predictor.")}, strict=True)
    joint.load_state_dict({k[len("joint."):]: v for k, v in sd.items() if k.startswith("joint.")}, strict=True)
    model = types.SimpleNamespace(predictor=pred, joint=joint, blank=0)
    g4 = np.load(os.path.join(HERE, "large_4h.npz"))
    starts = np.cumsum([0] + g4["nchunks"].tolist())
    utts = [torch.from_numpy(g4["out"][starts[u]: starts[u + 1]].reshape(-1, c.enc_dim)[: int(n)])
            for u, n in enumerate(g4["outlens"])]
    lens = torch.tensor([u.shape[0] for u in utts])
    enc_b = torch.nn.utils.rnn.pad_sequence(utts, batch_first=True)
    with torch.no_grad():
        out_e = optimized_search(model, enc_e, torch.tensor([enc_e.shape[1]]), n_steps)
        out_b = optimized_search(model, enc_b, lens, n_steps)
        hyps_b = batch_greedy_search(model, enc_b, lens, n_steps)
    from oracle import rnnt_ref
    _, m_e = rnnt_ref.optimized_search(sd, c.num_layers, c.hidden, enc_e, [enc_e.shape[1]], n_steps)
    _, m_b = rnnt_ref.optimized_search(sd, c.num_layers, c.hidden, enc_b, lens, n_steps)
    for nm, o in (("endless", out_e), ("batch", out_b)):
        cnt = (o.reshape(-1, n_steps) != 0).sum(-1)
        nb = cnt[cnt > 0]
        print(f"rnnt memory {nm}: frames {cnt.numel()}, blank-first {float((cnt == 0).float().mean()):.2f}, "
              f"non-blank frames {nb.numel()}: 1-3 tokens {float(((nb >= 1) & (nb <= 3)).float().mean()):.2f}, "
              f"at the cap {float((nb == n_steps).float().mean()):.2f}")
    print(f"rnnt memory min top-2 margins: endless {m_e:.2e}, batch {m_b:.2e}")
    flat = [t for h in hyps_b for t in h]
    np.savez_compressed(path, seed=np.array(seed), n_steps=np.array(n_steps), vocab=np.array(c.vocab),
                        frame_dirs=frame_dirs.numpy(), frame_bias=frame_bias.numpy(),
                        tokens=np.array(tokens, np.int32), forget=np.array(MEMORY_FORGET),
                        suppress=np.array(MEMORY_SUPPRESS), endless_out=out_e.numpy().astype(np.int32),
                        batch_lens=lens.numpy().astype(np.int32), batch_out=out_b.numpy().astype(np.int32),
                        batch_hyp_lens=np.array([len(h) for h in hyps_b]), batch_hyps=np.array(flat, np.int32),
                        margin_endless=np.array(m_e), margin_batch=np.array(m_b))


if __name__ == "__main__":
    which = sys.argv[1:] or ["masks", "small", "large", "large_4h", "large_endless", "large_full", "text", "stream",
                             "endless_tbd", "rnnt", "rows_neq", "small256", "rnnt_sparse", "rnnt_memory", "autocast", "endless_tail", "tiny_batch", "tiny_padded",
                             "large_full_mixed", "chunk_by_chunk"]
    if "masks" in which:
        gen_masks(os.path.join(HERE, "masks.npz"))
    if "small" in which:
        gen_small(os.path.join(HERE, "small.npz"))
    if "large" in which:
        gen_large(os.path.join(HERE, "large.npz"))
    if "large_4h" in which:
        gen_large_4h(os.path.join(HERE, "large_4h.npz"))
    if "large_endless" in which:
        gen_large_endless(os.path.join(HERE, "large_endless.npz"))
    if "text" in which:
        gen_text(os.path.join(HERE, "text.json"))
    if "large_full" in which:
        gen_large_full(os.path.join(HERE, "large_full.npz"))
    if "stream" in which:
        gen_stream(os.path.join(HERE, "stream.npz"))
    if "endless_tbd" in which:
        gen_endless_tbd(os.path.join(HERE, "endless_tbd80.npz"))
    if "rows_neq" in which:
        gen_rows_neq(os.path.join(HERE, "rows_neq.npz"))
    if "rnnt" in which:
        gen_rnnt(os.path.join(HERE, "rnnt.npz"))
    if "small256" in which:
        gen_small256(os.path.join(HERE, "small256.npz"))
    if "rnnt_sparse" in which:
        gen_rnnt_sparse(os.path.join(HERE, "rnnt_sparse.npz"))
    if "rnnt_memory" in which:
        gen_rnnt_memory(os.path.join(HERE, "rnnt_memory.npz"))
    if "autocast" in which:
        gen_autocast(os.path.join(HERE, "autocast.npz"))
    if "endless_tail" in which:
        gen_endless_tail(os.path.join(HERE, "endless_tail.npz"))
    if "tiny_batch" in which:
        gen_tiny_batch(os.path.join(HERE, "tiny_batch.npz"))
    if "tiny_padded" in which:
        gen_tiny_padded(os.path.join(HERE, "tiny_padded.npz"))
    if "chunk_by_chunk" in which:
        gen_chunk_by_chunk(os.path.join(HERE, "chunk_by_chunk.npz"))
    if "large_full_mixed" in which:
        gen_large_full_mixed(os.path.join(HERE, "large_full_mixed.npz"))
    print("ok", which)
