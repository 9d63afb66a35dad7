"""Host-side mirror of the reference `ChunkFormerModel` callers of the encoder hot path
(chunkformer/chunkformer_model.py), on top of `ChunkFormerEncoder` (libcfm.so):

  encode           chunkformer_model.py:256-274   padded batch -> (xs, xs_lens)
  endless_decode   chunkformer_model.py:321-459   segment loop with att/cnn caches carried
  batch_decode     chunkformer_model.py:462-552   duration-budget grouping -> masked batch -> CTC
  from_pretrained  chunkformer_model.py:107-200   LOCAL directory only (no hub access)

Audio (`_load_audio_and_extract_features`, 276-318): wherever the reference takes an
`audio_path`, this mirror takes a 16-bit PCM `.wav` path (decoded with the standard library,
features by the GPU Kaldi fbank of fbank.py with the reference's parameters, config
`fbank_conf` / `resample_conf`), or 80-dim fbank features directly -- a `[T, 80]` tensor, or a
path to a `.npy` (loaded with allow_pickle=False) / `.pt` (torch.load weights_only=True) file.

CTC post-processing (remove_duplicates_and_blank and get_output_with_timestamps' sentence
split, chunkformer/utils/model_utils.py:23-221) runs on the device (cfm_ctc_collapse); only
the id -> text mapping (class2str) and the hh:mm:ss:ms formatting stay on the host, so
`char_dict` models return strings like the reference.

`model: transducer` checkpoints (config.yaml, init_model.py:118-135) decode with the RNN-T greedy
search on the device (transducer.py, cfm_rnnt_greedy) exactly where the reference calls
optimized_search / batch_greedy_search (chunkformer_model.py:439-448, 533-543); their per-frame
decisions [T, n_steps] go through get_output_with_timestamps' transducer branch (no collapse).
`model: classification` checkpoints are out of scope and refused.
"""
from __future__ import annotations

import json
import math
import os
from typing import Dict, List, Optional, Sequence, Union

import numpy as np
import torch

from .config import EncoderConfig
from .encoder import ChunkFormerEncoder
from .streaming import EndlessGraphPipeline, EndlessGraphRunner, EndlessPipeline
from .transducer import RNNTConfig, RNNTGreedy

Features = Union[torch.Tensor, np.ndarray, str]


# ----------------------------------------------------------------------------- text helpers
def remove_duplicates_and_blank(hyp: Sequence[int], blank_id: int = 0) -> List[int]:
    """model_utils.py:23-32: collapse repeats, then drop blanks."""
    out: List[int] = []
    prev = None
    for t in hyp:
        t = int(t)
        if t != prev and t != blank_id:
            out.append(t)
        prev = t
    return out


def class2str(target: Sequence[int], char_dict: Dict[int, str]) -> str:
    """model_utils.py:135-139."""
    return "".join(char_dict[int(w)] for w in target).replace("▁", " ")


def get_output(hyps, char_dict: Dict[int, str]) -> List[str]:
    """model_utils.py:164-171 (asr_model branch)."""
    return [class2str(remove_duplicates_and_blank([int(t) for t in h]), char_dict).strip() for h in hyps]


def milliseconds_to_hhmmssms(ms: int) -> str:
    """model_utils.py:142-161."""
    h, rem = divmod(int(ms), 3600 * 1000)
    m, rem = divmod(rem, 60 * 1000)
    s, rem = divmod(rem, 1000)
    return f"{h:02}:{m:02}:{s:02}:{rem:03}"


def max_silence_frames(max_silence_duration: float) -> int:
    """model_utils.py:176: max_silence = max_silence_duration // 0.08 (80 ms frames); a negative
    value never closes a sentence, i.e. one segment per utterance."""
    ms = max_silence_duration // 0.08
    return int(ms) if ms >= 0 else 1 << 30


def format_segments(segs, char_dict: Dict[int, str]) -> List[dict]:
    """Device segments (tokens, start frame, end frame) -> the reference's items
    {"decode", "start", "end"} (model_utils.py:203-218: class2str(...).strip(), 80 ms frames)."""
    return [{"decode": class2str(toks, char_dict).strip(), "start": milliseconds_to_hhmmssms(st * 80),
             "end": milliseconds_to_hhmmssms(en * 80)} for toks, st, en in segs]


def transducer_segments(dense, max_silence: int):
    """get_output_with_timestamps (model_utils.py:174-221) for model_type "transducer": dense
    per-frame decisions [T, n_steps] (0 = blank; a frame is silent when all are blank, its tokens
    are the non-blank decisions in step order, no duplicate removal) -> [(tokens, start, end)] in
    80 ms frames.  Walks the non-blank frames only (a blank run closes the sentence when it
    reaches max_silence frames)."""
    d = np.asarray(dense)
    T = d.shape[0]
    nbf = np.nonzero((d != 0).any(1))[0].tolist()
    segs, toks, start, prev_end = [], [], -1, -1
    for i, t in enumerate(nbf):
        if start == -1:
            start = max(math.ceil((t + prev_end) / 2), t - 2) if prev_end != -1 else max(t - 2, 0)
        row = d[t]
        toks.extend(int(v) for v in row[row != 0])
        gap = (nbf[i + 1] if i + 1 < len(nbf) else T) - t - 1   # blank frames after t
        end = t if max_silence == 0 else (t + max_silence if 0 < max_silence <= gap else -1)
        if end != -1:
            segs.append((toks, start, end))
            prev_end, toks, start = end, [], -1
    if start != -1 and toks:
        segs.append((toks, start, T - 1))
    return segs


# ----------------------------------------------------------------------------- segment math
def endless_segments(xs_len: int, C: int, L: int, R: int, total_batch_duration: float, num_blocks: int,
                     kernel_size: int = 15, subsampling: int = 8):
    """The segment schedule of endless_decode (chunkformer_model.py:355-435) as plain
    integers: returns (truncated_context_size, [(start, stop, keep_trunc, last), ...]) where
    frames [start, stop) feed one forward_parallel_chunk call and `keep_trunc` says whether
    only the first `truncated_context_size` output frames are kept."""
    lorder = kernel_size // 2
    max_len = int(total_batch_duration // 0.01) // 2
    mult = max_len // C // subsampling
    trunc = C * mult
    if trunc <= 0:
        raise ValueError("total_batch_duration too small for one chunk")
    r = max(R, lorder)
    rel_right = (r + max(C, r) * (num_blocks - 1)) * subsampling
    step = trunc * subsampling
    segs = []
    for idx in range((xs_len + step - 1) // step if xs_len > 0 else 0):
        start = step * idx
        end = min(step * (idx + 1) + 7, xs_len)
        stop = min(end + rel_right, xs_len)
        last = step * idx + rel_right >= xs_len
        segs.append((start, stop, not last, last))
        if last:
            break
    return trunc, segs


def budget_groups(lens: Sequence[int], total_batch_duration: float) -> List[List[int]]:
    """batch_decode's grouping (chunkformer_model.py:481-529): utterances are appended
    until the frame budget int(tbd // 0.01) // 2 is used up (the utterance that crosses
    it is included), then the group is flushed; the tail is flushed at the end."""
    budget = int(total_batch_duration // 0.01) // 2
    groups, cur, left = [], [], budget
    for i, t in enumerate(lens):
        cur.append(i)
        left -= int(t)
        if left <= 0 or i == len(lens) - 1:
            groups.append(cur)
            cur, left = [], budget
    return groups


def _load_features(x: Features, featurize=None) -> torch.Tensor:
    if isinstance(x, str) and x.lower().endswith(".wav"):
        from .fbank import load_wav
        samples, sr = load_wav(x)
        return featurize(samples, sr)
    if isinstance(x, torch.Tensor):
        t = x
    elif isinstance(x, np.ndarray):
        t = torch.from_numpy(x)
    elif isinstance(x, str):
        if x.endswith(".npy"):
            t = torch.from_numpy(np.load(x, allow_pickle=False))
        elif x.endswith(".pt"):
            t = torch.load(x, map_location="cpu", weights_only=True)
        else:
            raise ValueError(f"{x}: only 16-bit PCM .wav audio is decoded here (no pydub/ffmpeg); or pass "
                             "80-dim fbank features ([T, 80] tensor, .npy or .pt)")
    else:
        raise TypeError(f"unsupported feature input {type(x)}")
    if t.dim() == 3 and t.shape[0] == 1:
        t = t[0]
    if t.dim() != 2:
        raise ValueError(f"features must be [T, F], got {tuple(t.shape)}")
    return t.float()


# ----------------------------------------------------------------------------- model
class ChunkFormerModel:
    """encoder + CTC head; the inference API of chunkformer_model.py on libcfm."""

    def __init__(self, cfg: EncoderConfig, state_dict: Dict[str, torch.Tensor], dtype: str = "bf16", device=None,
                 char_dict: Optional[Dict[int, str]] = None, fbank_conf: Optional[dict] = None,
                 resample_conf: Optional[dict] = None, model_type: str = "asr_model",
                 rnnt_config: Optional[RNNTConfig] = None):
        if model_type not in ("asr_model", "transducer"):
            raise AssertionError(f"model: {model_type} is out of scope (asr_model / transducer decoders only)")
        self.config = cfg
        self.model_type = model_type
        self.encoder = ChunkFormerEncoder(cfg, state_dict, device=device, dtype=dtype)
        self.device = self.encoder.device
        self.rnnt = None
        if model_type == "transducer":
            rc = rnnt_config or RNNTConfig(vocab=cfg.vocab, enc_dim=cfg.d_model)
            self.rnnt = RNNTGreedy(rc, state_dict, self.device)
        self.char_dict = char_dict
        self.fbank_conf = dict(fbank_conf or {})
        self.resample_conf = dict(resample_conf or {})
        self._fbank = None
        self._endless_runners: Dict[tuple, EndlessGraphRunner] = {}
        # endless_decode: truncated segments compute only the rows their kept rows depend on (native
        # "trim_right"; the kept rows, ids and caches are unchanged -- test_endless_trim_equals_full)
        self.endless_trim = True
        # endless_decode's graph pipeline: a segment's first front-end windows (the previous segment's last
        # complete ones, the same frames) are carried over instead of recomputed (streaming.py; exact)
        self.endless_fe_reuse = True

    def extract_features(self, samples, sample_rate: Optional[int] = None) -> torch.Tensor:
        """_load_audio_and_extract_features (chunkformer_model.py:276-318) after decoding:
        kaldi.fbank with the config's num_mel_bins / frame_length / frame_shift, dither 0,
        energy_floor 0, at resample_conf.resample_rate (16 kHz), on int16-scale samples; on the GPU."""
        rate = int(self.resample_conf.get("resample_rate", 16000))
        if sample_rate is not None and int(sample_rate) != rate:
            raise ValueError(f"audio at {sample_rate} Hz: resampling is not part of this build, expected {rate} Hz")
        if self._fbank is None:
            from .fbank import KaldiFbank
            self._fbank = KaldiFbank(self.device, num_mel_bins=int(self.fbank_conf.get("num_mel_bins", 80)),
                                     frame_length=float(self.fbank_conf.get("frame_length", 25)),
                                     frame_shift=float(self.fbank_conf.get("frame_shift", 10)), dither=0.0,
                                     energy_floor=0.0, sample_frequency=float(rate))
        return self._fbank(torch.as_tensor(samples, dtype=torch.float32))

    # ---------------------------------------------------------------- loading
    @classmethod
    def from_pretrained(cls, path: str, dtype: str = "bf16", device=None) -> "ChunkFormerModel":
        """Local checkpoint directory in the reference layout (chunkformer_model.py:107-200):

        * config.yaml (yaml.safe_load): encoder_conf, input_dim, output_dim, cmvn / cmvn_conf;
        * global_cmvn: JSON {mean_stat, var_stat, frame_num} or kaldi text stats
          (cmvn_conf.is_json_cmvn, utils/cmvn.py:23-98), used when config `cmvn: global_cmvn`
          (init_model.py:63-69);
        * pytorch_model.{bin,pt,ckpt} (torch.load weights_only=True: plain tensors only), loaded
          like load_checkpoint(strict=False) (checkpoint.py:26-41): keys present in the
          checkpoint win, so its `encoder.global_cmvn.{mean,istd}` buffers override the stats file
          exactly as load_state_dict does in the reference; model.safetensors is also accepted;
        * vocab.txt ("token id" per line, file_utils.py:62-69) -> char_dict for text output.
        There is no hub access: `path` must be a local directory."""
        import yaml
        if not os.path.isdir(path):
            raise FileNotFoundError(f"{path}: only local checkpoint directories are supported (no hub access)")
        cfg_path = os.path.join(path, "config.yaml")
        if not os.path.exists(cfg_path):
            raise ValueError(f"No config found in {path}")
        with open(cfg_path) as f:
            conf = yaml.safe_load(f)
        st = os.path.join(path, "model.safetensors")
        if os.path.exists(st):
            from safetensors.torch import load_file
            sd: Dict[str, torch.Tensor] = dict(load_file(st))
        else:
            cands = ["pytorch_model.bin", "pytorch_model.pt", "pytorch_model.ckpt"]
            for nm in cands:
                p = os.path.join(path, nm)
                if os.path.exists(p):
                    sd = torch.load(p, map_location="cpu", weights_only=True)
                    break
            else:
                raise ValueError(f"No checkpoint found in {path}. Expected one of: {cands}")
        # chunkformer_model.py:153-160, 91-100: GlobalCMVN exists exactly when the directory holds a
        # global_cmvn file (whatever config.yaml's `cmvn` key says), JSON unless the config's top-level
        # is_json_cmvn is false
        cmvn_path = os.path.join(path, "global_cmvn")
        has_cmvn = os.path.exists(cmvn_path)
        if has_cmvn:
            is_json = bool(conf.get("is_json_cmvn", True))
            mean, istd = load_json_cmvn(cmvn_path) if is_json else load_kaldi_cmvn(cmvn_path)
            sd.setdefault("encoder.global_cmvn.mean", torch.tensor(mean, dtype=torch.float64).float())
            sd.setdefault("encoder.global_cmvn.istd", torch.tensor(istd, dtype=torch.float64).float())
        else:   # no GlobalCMVN module: checkpoint buffers would be unexpected keys (ignored)
            sd.pop("encoder.global_cmvn.mean", None)
            sd.pop("encoder.global_cmvn.istd", None)
        model_type = conf.get("model", "asr_model")   # ChunkFormerConfig default (chunkformer_model.py:47-48)
        vocab = int(conf.get("output_dim", sd["ctc.ctc_lo.weight"].shape[0] if "ctc.ctc_lo.weight" in sd else 0))
        cfg = EncoderConfig.from_encoder_conf(conf.get("encoder_conf", {}), input_dim=int(conf.get("input_dim", 80)),
                                              output_dim=vocab, cmvn=has_cmvn)
        rnnt_cfg = RNNTConfig.from_conf(conf, vocab, cfg.d_model) if model_type == "transducer" else None
        char_dict = None
        vp = os.path.join(path, "vocab.txt")
        if os.path.exists(vp):
            char_dict = {}
            with open(vp, encoding="utf8") as f:
                for line in f:
                    arr = line.strip().split()
                    if len(arr) != 2:
                        raise AssertionError(f"bad vocab line {line!r}")
                    char_dict[int(arr[1])] = arr[0]
        return cls(cfg, sd, dtype=dtype, device=device, char_dict=char_dict, fbank_conf=conf.get("fbank_conf"),
                   resample_conf=conf.get("resample_conf"), model_type=model_type, rnnt_config=rnnt_cfg)

    # ---------------------------------------------------------------- API
    def encode(self, xs: torch.Tensor, xs_lens: torch.Tensor, chunk_size: Optional[int] = None,
               left_context_size: Optional[int] = None, right_context_size: Optional[int] = None, **kwargs):
        """chunkformer_model.py:256-274."""
        out, masks = self.encoder.forward_encoder(xs, xs_lens, chunk_size or 0, left_context_size or 0,
                                                  right_context_size or 0)
        return out, masks.squeeze(1).sum(-1)

    @torch.no_grad()
    def endless_decode(self, audio_path: Features, chunk_size: Optional[int] = 64,
                       left_context_size: Optional[int] = 128, right_context_size: Optional[int] = 128,
                       total_batch_duration: int = 1800, return_timestamps: bool = True,
                       max_silence_duration: float = 0.5, return_encoder_out: bool = False,
                       cuda_graph: bool = True, pipeline: Optional[bool] = None,
                       pipeline_depth: Optional[int] = None):
        """chunkformer_model.py:321-459.  Segments of `total_batch_duration` seconds (halved,
        like the reference) go through forward_parallel_chunk with the attention/conv caches
        and `offset` carried; the CTC argmax runs per segment on the kept rows (row-wise, so
        identical to the reference's argmax over the concatenation).
        Returns text (with char_dict) or ids [1, T', 1] like the reference; with
        `return_encoder_out` also the concatenated encoder output [1, T', d] (fp32).
        `pipeline` (default: on from 3 segments up): `pipeline_depth` (default 4 with graphs, 3 eager:
        the measured best of each at tbd 1800) segments in flight on as many
        streams, segment k + 1's layer l waiting only for segment k's layer l; with `cuda_graph` all
        segments (up to 128 per graph) replay one captured HIP graph of that whole multi-stream pipeline
        (EndlessGraphPipeline), without it every call is launched eagerly (EndlessPipeline).  pipeline=False: one segment at a time, the full-size
        middle segments replaying one captured graph (EndlessGraphRunner) when `cuda_graph`.  Every
        mode gives the same result as the eager loop (same kernels, same plans); see streaming.py."""
        C = chunk_size if chunk_size is not None else 64
        L = left_context_size if left_context_size is not None else 128
        R = right_context_size if right_context_size is not None else 128
        cfg, enc, dev = self.config, self.encoder, self.device
        xs = _load_features(audio_path, self.extract_features)
        trunc, segs = endless_segments(xs.shape[0], C, L, R, total_batch_duration, cfg.num_blocks, cfg.kernel_size)
        xs_dev = xs.to(dev, torch.float32)
        ids, outs = [], []
        seg_len = max(stop - start for start, stop, _, _ in segs) if segs else 0
        transducer = self.model_type == "transducer"
        want_eo = bool(return_encoder_out) or transducer   # the RNN-T search consumes the encoder rows
        if pipeline is None:
            pipeline = len(segs) >= 3
        if pipeline_depth is None:
            pipeline_depth = 4 if cuda_graph else 3
        trim = bool(self.endless_trim)
        fe_reuse = bool(self.endless_fe_reuse)
        key = (C, L, R, trunc, seg_len, want_eo, bool(cuda_graph), bool(pipeline), int(pipeline_depth), trim, fe_reuse)
        runner = self._endless_runners.get(key)
        if runner is None:   # graphs are captured once per segment geometry and reused across calls
            for old in self._endless_runners.values():   # the replaced runner's graphs are destroyed
                old.close()
            self._endless_runners = {}
            if pipeline:
                runner = (EndlessGraphPipeline(enc, C, L, R, trunc, seg_len, want_eo, pipeline_depth, trim=trim,
                                               fe_reuse=fe_reuse)
                          if cuda_graph else EndlessPipeline(enc, C, L, R, trunc, want_eo, pipeline_depth, trim=trim))
            else:
                runner = EndlessGraphRunner(enc, C, L, R, trunc, seg_len, want_eo, use_graph=cuda_graph, trim=trim)
            self._endless_runners = {key: runner}
        if pipeline:
            tids, teos, cur = runner.run(xs_dev, segs)
            ids = [t for t in tids if t is not None]
            outs = [e for e in teos if e is not None]
            self.last_endless_caches = (runner.att[cur], runner.cnn[cur])
        else:
            runner.reset()
            offset = 0
            try:
                for start, stop, keep_trunc, _ in segs:
                    # forward_parallel_chunk with att/cnn caches carried; offset += len, then -= dropped rows
                    tok, eo, kept = runner.step(xs_dev[start:stop], offset, keep_trunc)
                    offset += kept
                    if tok is not None:
                        ids.append(tok)
                    if eo is not None:
                        outs.append(eo)
            finally:
                enc._set_trim(False)
            # the caches carried out of the last segment (r_att_cache / r_cnn_cache of its
            # forward_parallel_chunk call, chunkformer_model.py:407-417)
            self.last_endless_caches = (runner.att[runner.cur], runner.cnn[runner.cur])
        if transducer:
            # optimized_search over the concatenated encoder output (chunkformer_model.py:439-448):
            # decisions [1, T, n_steps], text by get_output_with_timestamps' transducer branch
            enc_all = torch.cat(outs) if outs else torch.zeros(0, cfg.d_model, device=dev)
            T = enc_all.shape[0]
            dense = self.rnnt.greedy_packed(enc_all, [0], [T])
            tokens = dense.long().reshape(1, T, -1)
            if self.char_dict is not None:
                segs_t = transducer_segments(dense.cpu().numpy(), max_silence_frames(max_silence_duration))
                res = format_segments(segs_t, self.char_dict)
                if not return_timestamps:
                    res = " ".join(item["decode"] for item in res).strip()
            else:
                res = tokens
            if return_encoder_out:
                return res, enc_all.unsqueeze(0)
            return res
        tokens = torch.cat(ids).long().reshape(1, -1, 1) if ids else None
        if self.char_dict is not None and tokens is not None:
            # get_output_with_timestamps (model_utils.py:174-221) on the device: sentence split at
            # max_silence blank frames, de-duplicated tokens per sentence
            segs = enc.ctc_collapse(tokens, [0], [tokens.shape[1]],
                                    max_silence=max_silence_frames(max_silence_duration))[0]
            res = format_segments(segs, self.char_dict)
            if not return_timestamps:
                res = " ".join(item["decode"] for item in res).strip()
        else:
            res = tokens
        if return_encoder_out:
            return res, torch.cat(outs).unsqueeze(0)
        return res

    @torch.no_grad()
    def batch_decode(self, audio_paths: List[Features], chunk_size: Optional[int] = 64,
                     left_context_size: Optional[int] = 128, right_context_size: Optional[int] = 128,
                     total_batch_duration: int = 1800):
        """chunkformer_model.py:462-552 (asr_model branch): budget grouping, one masked-batch
        encoder call per group, CTC argmax, per-utterance split to its subsampled length."""
        C = chunk_size if chunk_size is not None else 64
        L = left_context_size if left_context_size is not None else 128
        R = right_context_size if right_context_size is not None else 128
        feats = [_load_features(a, self.extract_features) for a in audio_paths]
        decodes = []
        for grp in budget_groups([f.shape[0] for f in feats], total_batch_duration):
            xs = [feats[i] for i in grp]
            lens = torch.tensor([x.shape[0] for x in xs], dtype=torch.int)
            offset = torch.zeros(len(xs), dtype=torch.int)
            eo, el, n_chunks, _, _, _ = self.encoder.forward_parallel_chunk(xs, lens, C, L, R, offset=offset)
            # per-utterance rows as the reference slices them: hyp.flatten()[:x_len] (Python slice: an
            # utterance under 7 frames has calc_length -1 and keeps all but the last row of its padded
            # chunk) and, for the transducer, frames t < encoder_out_lens (none at <= 0)
            el_ctc = [len(range(int(nc) * C)[: int(n)]) for nc, n in zip(n_chunks, el.tolist())]
            el_rnnt = [max(0, int(n)) for n in el.tolist()]
            if self.model_type == "transducer":
                # batch_greedy_search over each utterance's rows (chunkformer_model.py:533-543): the
                # packed rows go straight in (no pad_sequence), one workgroup per utterance
                starts = (np.cumsum([0] + list(n_chunks[:-1])) * C).tolist()
                dense = self.rnnt.greedy_packed(eo.reshape(-1, eo.shape[-1]), starts, el_rnnt).cpu()
                hyps = [dense[s0: s0 + n].reshape(-1) for s0, n in zip(starts, el_rnnt)]
                hyps = [h[h != self.rnnt.cfg.blank].tolist() for h in hyps]
                if self.char_dict is not None:
                    decodes.extend(class2str(h, self.char_dict).strip() for h in hyps)
                else:
                    decodes.extend(hyps)
                continue
            _, hyp = self.encoder.ctc_log_softmax(eo, want_logp=False)   # fused argmax head
            if self.char_dict is not None:
                # remove_duplicates_and_blank on the device, per utterance rows [64 * chunk0, +len)
                starts = np.cumsum([0] + list(n_chunks[:-1])) * C
                toks = self.encoder.ctc_collapse(hyp, starts.tolist(), el_ctc)
                decodes.extend(class2str(t, self.char_dict).strip() for t, _ in toks)
            else:
                decodes.extend(h.flatten()[:n].long() for h, n in zip(hyp.split(n_chunks, dim=0), el_ctc))
        return decodes


def _cmvn_from_stats(mean_stat, var_stat, count):
    mean = [m / count for m in mean_stat]
    istd = []
    for m, v in zip(mean, var_stat):
        var = v / count - m * m
        if var < 1.0e-20:
            var = 1.0e-20
        istd.append(1.0 / math.sqrt(var))
    return mean, istd


def load_json_cmvn(path: str):
    """utils/cmvn.py:23-45: JSON {mean_stat, var_stat, frame_num} -> (mean, istd)."""
    with open(path) as f:
        st = json.load(f)
    return _cmvn_from_stats(st["mean_stat"], st["var_stat"], st["frame_num"])


def load_kaldi_cmvn(path: str):
    """utils/cmvn.py:48-90: kaldi text stats `[ m_1 .. m_F count v_1 .. v_F 0 ]` -> (mean, istd);
    the binary kaldi form is rejected like the reference."""
    with open(path, "r") as f:
        if f.read(2) == "\0B":
            raise ValueError("kaldi cmvn binary file is not supported; recompute it with "
                             "compute-cmvn-stats --binary=false")
        f.seek(0)
        arr = f.read().split()
    if not (arr[0] == "[" and arr[-2] == "0" and arr[-1] == "]"):
        raise AssertionError(f"{path}: not a kaldi text cmvn file")
    F = (len(arr) - 4) // 2
    means = [float(a) for a in arr[1: F + 1]]
    count = float(arr[F + 1])
    var = [float(a) for a in arr[F + 2: 2 * F + 2]]
    return _cmvn_from_stats(means, var, count)
