"""Host-side mirror of the reference `ChunkFormerEncoder` (chunkformer/modules/encoder.py).

Same method names, argument meaning, return tuples and error types as the
reference; every tensor op of the hot path runs in libcfm.so (HIP, gfx950):

  forward_parallel_chunk  encoder.py:503-681   -> cfm_plan_masked + cfm_encode_masked_utts
  forward_encoder         encoder.py:220-274   -> cfm_plan_padded + cfm_encode_padded
  forward                 encoder.py:461-501   (eval branch: negative sizes -> 0/0/0)
  forward_chunk           encoder.py:310-385   -> cfm_plan_stream + cfm_encode_stream (realtime path)
  ctc_log_softmax/argmax  ctc.py:73-91          -> cfm_ctc_logprobs / cfm_ctc_ids (fused argmax)
  ctc_collapse            model_utils.py:23-58, 174-221 -> cfm_ctc_collapse

Python only moves pointers: it builds the host plan (C++ planner), uploads it,
allocates outputs/workspace with torch on the current device and launches on
torch's current stream.
"""
from __future__ import annotations

import contextlib
import ctypes
import weakref
from typing import Dict, List, Optional, Tuple

import torch

from . import _lib
from .config import EncoderConfig
from .weights import check_state_dict

_DTYPES = {"fp32": _lib.DTYPE_F32, "float32": _lib.DTYPE_F32, "bf16": _lib.DTYPE_BF16, "bfloat16": _lib.DTYPE_BF16,
           "fp16": _lib.DTYPE_F16, "float16": _lib.DTYPE_F16}


def calc_length(T: int) -> int:
    """subsampling.py:270-288 (integer form)."""
    return 1 + (int(T) - 15) // 8


def reverse_calc_length(out_len: int) -> int:
    """subsampling.py:290-311: the input length that subsamples to out_len (three kernel-3, stride-2
    stages without padding: n -> 2 (n - 1) + 3 each, i.e. 8 (out_len - 1) + 15); 0 for out_len <= 0."""
    if out_len <= 0:
        return 0
    n = int(out_len)
    for _ in range(3):
        n = (n - 1) * 2 + 3
    return n


class ChunkFormerEncoder:
    subsampling_rate = 8
    right_context = 14

    def __init__(self, cfg: EncoderConfig, state_dict: Dict[str, torch.Tensor], device=None, dtype: str = "bf16"):
        cfg.validate()
        check_state_dict(cfg, state_dict)
        if not torch.cuda.is_available():
            raise RuntimeError("chunkformer_amd needs a ROCm GPU (MI355X); there is no CPU fallback")
        self.cfg = cfg
        self.device = torch.device(device) if device is not None else torch.device("cuda", torch.cuda.current_device())
        if dtype not in _DTYPES:
            raise ValueError(f"dtype must be one of {list(_DTYPES)}")
        self.dtype = {_lib.DTYPE_F32: "fp32", _lib.DTYPE_BF16: "bf16", _lib.DTYPE_F16: "fp16"}[_DTYPES[dtype]]
        self.num_blocks = cfg.num_blocks
        self.attention_heads = cfg.n_heads
        self._output_size = cfg.d_model
        self.cnn_module_kernel = cfg.kernel_size
        c = _lib.CfmConfig(cfg.input_dim, cfg.d_model, cfg.n_heads, cfg.ffn_dim, cfg.num_blocks, cfg.kernel_size,
                           cfg.vocab, cfg.norm_eps, int(cfg.cmvn), _DTYPES[dtype])
        keep = []
        views = (_lib.CfmTensorView * len(state_dict))()
        for i, (k, v) in enumerate(state_dict.items()):
            t = v.detach().to("cpu", torch.float32).contiguous()
            keep.append(t)
            views[i] = _lib.CfmTensorView(k.encode(), t.data_ptr(), t.numel())
        h = ctypes.c_void_p()
        with torch.cuda.device(self.device):
            _lib.check(_lib.cfm_model_create(ctypes.byref(c), views, len(state_dict), self.device.index or 0,
                                             ctypes.byref(h)))
        self._h = h
        self._ws: Optional[torch.Tensor] = None
        # option: large masked batches as `stream_split` utterance groups on as many streams, staggered
        # by encoder layer (_encode_masked_split); per-utterance results do not depend on the grouping.
        # Off by default: +1-2.6% frames/s on the 240-min batch, but each kernel then shares the chip
        # with the other group's, which hides its own roofline (FFN w1 0.37 ms -> 0.29 ms at half the rows)
        self.stream_split = 1
        self.split_min_chunks = 1024
        self._native_opts: dict = {}
        self._split_streams: List[torch.cuda.Stream] = []
        self._split_ws: List[Optional[torch.Tensor]] = []
        # destroy the native handle when this object is collected or at interpreter exit (a finalizer
        # holds its own reference to the bound ctypes function, unlike __del__ at shutdown)
        self._finalizer = weakref.finalize(self, _lib.cfm_model_destroy, ctypes.c_void_p(h.value))

    def output_size(self) -> int:
        return self._output_size

    def set_option(self, key: str, value: int) -> None:
        if key in ("stream_split", "split_min_chunks"):   # host-side scheduling knobs
            if int(value) < (1 if key == "stream_split" else 0):
                raise ValueError(f"{key} = {value}")
            setattr(self, key, int(value))
            return
        _lib.check(_lib.cfm_model_set_option(self._h, key.encode(), int(value)))
        self._native_opts[key] = int(value)

    # the native options' values before any set_option (csrc/cfm_kernels.h Tuning)
    _NATIVE_DEFAULTS = {"wsp_small_div": 1, "wsp_small_rows": 32768, "attn_min_chunks": 2,
                        "gemm_big_min": 0}

    @contextlib.contextmanager
    def scoped_options(self, **opts):
        """Native options for the duration of a with-block (launch parameters only: results are the
        same), then the previous values; options the caller set explicitly are left alone."""
        keep = {k: self._native_opts.get(k, self._NATIVE_DEFAULTS[k]) for k in opts}
        explicit = {k for k in opts if k in self._native_opts}
        for k, v in opts.items():
            if k not in explicit:
                _lib.check(_lib.cfm_model_set_option(self._h, k.encode(), int(v)))
        try:
            yield
        finally:
            for k in opts:
                if k not in explicit:
                    _lib.check(_lib.cfm_model_set_option(self._h, k.encode(), int(keep[k])))

    def _set_trim(self, on: bool) -> None:
        """Native "trim_right" for the next encode calls (endless_decode's truncated segments only: their
        rows past truncated_context_size are not computed -- the caller drops them)."""
        _lib.check(_lib.cfm_model_set_option(self._h, b"trim_right", int(bool(on))))

    def _set_fe_carry(self, ptr: int, reuse: int, save_from: int) -> None:
        """Native "fe_carry" / "fe_reuse" / "fe_save_from" for the next encode calls (endless_decode's
        pipelined segments): the first `reuse` front-end windows' output rows come from the f32 buffer at
        `ptr`, and the rows of windows [save_from, nwin) are copied into it (-1: none); ptr 0 = off."""
        _lib.check(_lib.cfm_model_set_option(self._h, b"fe_carry", int(ptr)))
        _lib.check(_lib.cfm_model_set_option(self._h, b"fe_reuse", int(reuse)))
        _lib.check(_lib.cfm_model_set_option(self._h, b"fe_save_from", int(save_from)))

    # ------------------------------------------------------------------ helpers
    def _workspace(self, nbytes: int) -> torch.Tensor:
        if self._ws is None or self._ws.numel() < nbytes:
            self._ws = None
            self._ws = torch.empty(nbytes, dtype=torch.uint8, device=self.device)
        return self._ws

    def _stream(self) -> int:
        return torch.cuda.current_stream(self.device).cuda_stream

    def _upload(self, plan: torch.Tensor) -> torch.Tensor:
        return plan.pin_memory().to(self.device, non_blocking=True)

    # ------------------------------------------------------------------ masked batch
    @torch.no_grad()
    def forward_parallel_chunk(self, xs, xs_origin_lens, chunk_size: int = -1, left_context_size: int = -1,
                               right_context_size: int = -1, att_cache: torch.Tensor = torch.zeros((0, 0, 0)),
                               cnn_cache: torch.Tensor = torch.zeros((0, 0)), truncated_context_size: int = 0,
                               offset: torch.Tensor = torch.zeros(0)):
        """encoder.py:503-681.  Returns (xs [N, C, d], xs_lens [B] int32, n_chunks, r_att_cache,
        r_cnn_cache, offset); `offset` is updated in place (+= xs_lens) like the reference."""
        B = len(xs)
        C, L, R = int(chunk_size), int(left_context_size), int(right_context_size)
        dev = self.device
        if offset.shape[0] == 0:
            offset = torch.zeros(B, dtype=torch.long, device=xs_origin_lens.device)
        mask_lens = [int(t) for t in xs_origin_lens.tolist()]
        if len(mask_lens) != B:
            raise ValueError(f"{B} utterances but {len(mask_lens)} xs_origin_lens")
        # the reference pads / unfolds x.size(0) rows (encoder.py:556-564) and bounds the masks and the
        # output lengths by xs_origin_lens (567-596, 673); the planner takes both
        lens = [x.reshape(-1, self.cfg.input_dim).shape[0] for x in xs]
        offs = [int(o) for o in offset.tolist()]
        plan, n_chunks, out_lens = _lib.plan_masked(lens, offs, C, L, R,
                                                    mask_lens=None if lens == mask_lens else mask_lens)
        N = sum(n_chunks)
        d = self.cfg.d_model
        # the utterances are read where they are (cfm_encode_masked_utts: a device table of B row
        # pointers), not concatenated first; only inputs that are not already f32 on this device are copied
        utts = [x.to(dev, torch.float32).reshape(-1, self.cfg.input_dim).contiguous() for x in xs]
        out = torch.empty(N * C, d, dtype=torch.float32, device=dev)
        has_cache = att_cache.size(0) > 0
        aci = cci = aco = cco = None
        if has_cache:
            nb = self.num_blocks
            aci = att_cache.to(dev, torch.float32).contiguous()
            cci = cnn_cache.to(dev, torch.float32).contiguous()
            if tuple(aci.shape) != (nb, L, self.cfg.n_heads, 2 * self.cfg.head_dim):
                raise ValueError(f"att_cache shape {tuple(aci.shape)} != {(nb, L, self.cfg.n_heads, 2 * self.cfg.head_dim)}")
            if tuple(cci.shape) != (nb, d, self.cfg.conv_lorder):
                raise ValueError(f"cnn_cache shape {tuple(cci.shape)} != {(nb, d, self.cfg.conv_lorder)}")
            aco = torch.empty_like(aci)
            cco = torch.empty_like(cci)
        parts = min(self.stream_split, B)
        if not has_cache and parts > 1 and N >= self.split_min_chunks:
            feats = torch.cat(utts, 0)
            self._encode_masked_split(feats, lens, offs, mask_lens, n_chunks, parts, C, L, R, out)
        else:
            plan_dev = self._upload(plan)
            ws_bytes = _lib.cfm_workspace_bytes_masked(self._h, N, C, L, R)
            ws = self._workspace(ws_bytes)
            # an empty utterance still needs a readable row pointer (its windows read no rows)
            tab = self._upload(torch.tensor([u.data_ptr() if u.numel() else out.data_ptr() for u in utts],
                                            dtype=torch.int64))
            # the uploaded plan, pointer table and utterance tensors stay alive until the stream consumed them
            self._last_plan = (plan, plan_dev, tab, utts)
            _lib.check(_lib.cfm_encode_masked_utts(self._h, tab.data_ptr(), plan.data_ptr(), plan_dev.data_ptr(),
                                                   _lib.ptr(aci), _lib.ptr(cci), int(truncated_context_size),
                                                   _lib.ptr(aco), _lib.ptr(cco), out.data_ptr(), ws.data_ptr(),
                                                   ws_bytes, self._stream()))
        xs_lens = torch.tensor(out_lens, dtype=torch.int32, device=xs_origin_lens.device)
        offset += xs_lens.to(offset.device)
        if has_cache:
            r_att, r_cnn = aco, cco
        else:
            r_att = torch.zeros(self.num_blocks, 0, 0, 0, device=dev)
            r_cnn = torch.zeros(self.num_blocks, 0, 0, device=dev)
        return out.view(N, C, d), xs_lens, n_chunks, r_att, r_cnn, offset

    def _encode_masked_split(self, feats, lens, offs, mask_lens, n_chunks, parts, C, L, R, out) -> None:
        """The masked batch as `parts` groups of consecutive utterances (balanced by chunk count),
        group i on stream i: its front-end first, then encoder layer l once group i - 1 finished
        layer l (cfm_encode_masked_stages).  Each group writes its own rows of `out` (the batch's
        chunk order is utterance order), so the result is bit-identical to the single launch
        sequence: every kernel computes a row / chunk from that row's / chunk's inputs alone.  The
        groups' kernels overlap where a launch leaves CUs idle (tail rounds, the LayerNorm / GEMM
        boundaries): 240 min on one MI355X 50.9 -> 49.6 ms (tools/split_bench.py, 2 groups; 3 and 4
        groups gain less); in bench.py runs 50.3-50.5 -> 49.4-50.4 ms."""
        nb, dev = self.num_blocks, self.device
        total = sum(n_chunks)
        cuts, acc, k = [0], 0, 1
        for u, n in enumerate(n_chunks):
            acc += n
            if k < parts and acc >= total * k / parts and u + 1 < len(n_chunks):
                cuts.append(u + 1)
                k += 1
        cuts.append(len(n_chunks))
        cur = torch.cuda.current_stream(dev)
        while len(self._split_streams) < len(cuts) - 1:
            self._split_streams.append(torch.cuda.Stream(dev))
            self._split_ws.append(None)
        jobs, f0, c0 = [], 0, 0
        for i in range(len(cuts) - 1):
            a, b = cuts[i], cuts[i + 1]
            ls, ml = lens[a:b], mask_lens[a:b]
            plan, nc, _ = _lib.plan_masked(ls, offs[a:b], C, L, R, mask_lens=None if ls == ml else ml)
            n, F = sum(nc), sum(ls)
            wsb = int(_lib.cfm_workspace_bytes_masked(self._h, n, C, L, R))
            if self._split_ws[i] is None or self._split_ws[i].numel() < wsb:
                self._split_ws[i] = None
                self._split_ws[i] = torch.empty(wsb, dtype=torch.uint8, device=dev)
            jobs.append((plan, self._upload(plan), feats[f0: f0 + F], out[c0 * C: (c0 + n) * C], wsb, i))
            f0, c0 = f0 + F, c0 + n
        for i in range(len(jobs)):
            self._split_streams[i].wait_stream(cur)   # features, plans, output allocated on `cur`
        prev = None
        for plan, plan_dev, fe, o, wsb, i in jobs:
            st = self._split_streams[i]
            ws = self._split_ws[i]
            evs = []
            for stage in range(-1, nb):
                if stage >= 0 and prev is not None:
                    st.wait_event(prev[stage])
                _lib.check(_lib.cfm_encode_masked_stages(self._h, fe.data_ptr(), plan.data_ptr(), plan_dev.data_ptr(),
                                                         None, None, 0, None, None, o.data_ptr(), ws.data_ptr(), wsb,
                                                         stage, stage, st.cuda_stream))
                if stage >= 0:
                    e = torch.cuda.Event()
                    e.record(st)
                    evs.append(e)
            prev = evs
        for i in range(len(jobs)):
            cur.wait_stream(self._split_streams[i])
        self._last_split = [(j[0], j[1]) for j in jobs]   # uploaded plans stay alive until consumed

    def _encode_masked_raw(self, feats, plan, plan_dev, aci, cci, trunc, aco, cco, out, ws) -> None:
        """One cfm_encode_masked launch sequence on the current stream: no allocation and no host
        synchronisation, so it can be captured into a HIP graph (EndlessGraphRunner)."""
        C, L, R = (int(plan[i]) for i in (5, 6, 7))
        ws_bytes = _lib.cfm_workspace_bytes_masked(self._h, int(plan[1]), C, L, R)
        if ws.numel() < ws_bytes:
            raise ValueError(f"workspace {ws.numel()} B < {ws_bytes} B")
        _lib.check(_lib.cfm_encode_masked(self._h, feats.data_ptr(), plan.data_ptr(), plan_dev.data_ptr(),
                                          _lib.ptr(aci), _lib.ptr(cci), int(trunc), _lib.ptr(aco), _lib.ptr(cco),
                                          out.data_ptr(), ws.data_ptr(), ws_bytes, self._stream()))

    def ctc_ws_bytes(self, rows: int, want_logp: bool) -> int:
        """Workspace of the CTC head over `rows` rows: 0 for ids only on the fused argmax head."""
        if want_logp:
            return int(_lib.cfm_ctc_workspace_bytes(self._h, rows))
        return int(_lib.cfm_ctc_ids_workspace_bytes(self._h, rows))

    def _ctc_raw(self, enc: torch.Tensor, rows: int, logp, ids, ws) -> None:
        """CTC head over the first `rows` rows of enc [*, d] (graph-capturable): cfm_ctc_logprobs,
        or the fused ids-only cfm_ctc_ids when no log-probs are asked for."""
        nbytes = self.ctc_ws_bytes(rows, logp is not None)
        wsz = 0 if ws is None else ws.numel()
        if wsz < nbytes:
            raise ValueError(f"CTC workspace {wsz} B < {nbytes} B")
        wp = _lib.ptr(ws) if nbytes > 0 else None
        if logp is None:
            _lib.check(_lib.cfm_ctc_ids(self._h, enc.data_ptr(), rows, ids.data_ptr(), wp, nbytes, self._stream()))
        else:
            _lib.check(_lib.cfm_ctc_logprobs(self._h, enc.data_ptr(), rows, logp.data_ptr(), _lib.ptr(ids), wp,
                                             nbytes, self._stream()))

    @torch.no_grad()
    def masks(self, xs_origin_lens, chunk_size: int, left_context_size: int, right_context_size: int,
              offset: Optional[torch.Tensor] = None) -> Tuple[torch.Tensor, torch.Tensor]:
        """att_mask [N,1,L+C+R] and mask_pad [N,1,C+14] exactly as encoder.py:627-645 builds them."""
        lens = [int(t) for t in xs_origin_lens.tolist()]
        offs = [0] * len(lens) if offset is None or offset.shape[0] == 0 else [int(o) for o in offset.tolist()]
        C, L, R = chunk_size, left_context_size, right_context_size
        plan, n_chunks, _ = _lib.plan_masked(lens, offs, C, L, R)
        N = sum(n_chunks)
        plan_dev = self._upload(plan)
        att = torch.empty(N, L + C + R, dtype=torch.uint8, device=self.device)
        pad = torch.empty(N, C + 14, dtype=torch.uint8, device=self.device)
        _lib.check(_lib.cfm_masks_from_plan(plan.data_ptr(), plan_dev.data_ptr(), att.data_ptr(), pad.data_ptr(),
                                            self._stream()))
        torch.cuda.current_stream(self.device).synchronize()
        return att.bool().unsqueeze(1), pad.bool().unsqueeze(1)

    # ------------------------------------------------------------------ padded batch
    @torch.no_grad()
    def forward_encoder(self, xs: torch.Tensor, xs_lens: torch.Tensor, chunk_size: int = 0,
                        left_context_size: int = 0, right_context_size: int = 0):
        """encoder.py:220-274: padded [B, T, 80] -> ([B, T', d], masks [B, 1, T'] bool)."""
        B, T, F = xs.shape
        if F != self.cfg.input_dim:
            raise RuntimeError(f"expected {self.cfg.input_dim} input features, got {F}")
        lens = [int(t) for t in xs_lens.tolist()]
        plan, Tp = _lib.plan_padded(lens, T, int(chunk_size), int(left_context_size), int(right_context_size))
        dev = self.device
        x = xs.to(dev, torch.float32).contiguous()
        plan_dev = self._upload(plan)
        out = torch.empty(B, Tp, self.cfg.d_model, dtype=torch.float32, device=dev)
        ws_bytes = _lib.cfm_workspace_bytes_padded(self._h, B, T, int(chunk_size), int(left_context_size),
                                                   int(right_context_size))
        ws = self._workspace(ws_bytes)
        _lib.check(_lib.cfm_encode_padded(self._h, x.data_ptr(), plan.data_ptr(), plan_dev.data_ptr(), out.data_ptr(),
                                          ws.data_ptr(), ws_bytes, self._stream()))
        self._last_plan = (plan, plan_dev)
        sub = torch.tensor([calc_length(t) for t in lens], device=dev)
        masks = (torch.arange(Tp, device=dev)[None, :] < sub[:, None]).unsqueeze(1)
        return out, masks

    # ------------------------------------------------------------------ streaming
    @torch.no_grad()
    def forward_chunk(self, xs: torch.Tensor, att_cache: torch.Tensor = torch.zeros((0, 0, 0, 0, 0)),
                      cnn_cache: torch.Tensor = torch.zeros((0, 0, 0, 0)), chunk_size: int = 0,
                      left_context_size: int = 0, right_context_size: int = 0, offset: int = 0):
        """encoder.py:310-385: one streaming step of the realtime app (stream_asr.py:164-172).
        xs [B, T, 80]; att_cache [nb, B, H, L, 2dk], cnn_cache [nb, B, d, 7] (required; zeros at the
        stream start); returns (xs [B, T', d], None, new att_cache, new cnn_cache) like the reference
        (its second value is an unused placeholder)."""
        if xs.dim() != 3 or xs.shape[-1] != self.cfg.input_dim:
            raise RuntimeError(f"expected xs [B, T, {self.cfg.input_dim}], got {tuple(xs.shape)}")
        B, T, _ = xs.shape
        C, L, R = int(chunk_size), int(left_context_size), int(right_context_size)
        nb, H, dk, d = self.num_blocks, self.cfg.n_heads, self.cfg.head_dim, self.cfg.d_model
        if att_cache.dim() != 5 or att_cache.size(3) == 0:
            raise AssertionError("forward_chunk needs att_cache [num_blocks, B, H, left_context_size, 2*d_k] "
                                 "(zeros at the start of a stream)")
        if tuple(att_cache.shape) != (nb, B, H, L, 2 * dk):
            raise ValueError(f"att_cache shape {tuple(att_cache.shape)} != {(nb, B, H, L, 2 * dk)}")
        if tuple(cnn_cache.shape) != (nb, B, d, self.cfg.conv_lorder):
            raise ValueError(f"cnn_cache shape {tuple(cnn_cache.shape)} != {(nb, B, d, self.cfg.conv_lorder)}")
        plan, Tp = _lib.plan_stream(T, C, L, R, int(offset))
        dev = self.device
        x = xs.to(dev, torch.float32).contiguous()
        aci = att_cache.to(dev, torch.float32).contiguous()
        cci = cnn_cache.to(dev, torch.float32).contiguous()
        aco, cco = torch.empty_like(aci), torch.empty_like(cci)
        out = torch.empty(B, Tp, d, dtype=torch.float32, device=dev)
        plan_dev = self._upload(plan)
        ws_bytes = _lib.cfm_workspace_bytes_stream(self._h, T, C, L, R)
        ws = self._workspace(ws_bytes)
        _lib.check(_lib.cfm_encode_stream(self._h, x.data_ptr(), B, plan.data_ptr(), plan_dev.data_ptr(),
                                          aci.data_ptr(), cci.data_ptr(), aco.data_ptr(), cco.data_ptr(),
                                          out.data_ptr(), ws.data_ptr(), ws_bytes, self._stream()))
        self._last_plan = (plan, plan_dev)
        return out, None, aco, cco

    @torch.no_grad()
    def forward_chunk_by_chunk(self, xs: torch.Tensor, xs_lens: torch.Tensor, chunk_size: int = 0,
                               left_context_size: int = 0, right_context_size: int = 0):
        """encoder.py:387-459: streaming decode of a padded batch xs [B, T, 80] through forward_chunk, the
        caches carried: the input is padded so that (T - size) is a multiple of the stride (size =
        reverse_calc_length(chunk_size) + 8 right_context_size input frames per step, stride 8 chunk_size),
        every step keeps its first chunk_size rows but the last one keeps its whole output; returns
        (out [B, T', d], masks [B, 1, T']) with the masks of calc_length(xs_lens + pad) like the reference."""
        B = xs.size(0)
        C, L, R = int(chunk_size), int(left_context_size), int(right_context_size)
        nb, H, dk, d = self.num_blocks, self.cfg.n_heads, self.cfg.head_dim, self.cfg.d_model
        size = reverse_calc_length(C) + R * self.subsampling_rate
        stride = C * self.subsampling_rate
        if stride <= 0:
            raise ValueError("forward_chunk_by_chunk needs chunk_size > 0")
        pad = stride - ((xs.size(1) - size) % stride)
        xs = torch.nn.functional.pad(xs, (0, 0, 0, pad))
        lens = torch.as_tensor(xs_lens) + pad
        dev = self.device
        att = torch.zeros(nb, B, H, L, 2 * dk, device=dev)
        cnn = torch.zeros(nb, B, d, self.cfg.conv_lorder, device=dev)
        outs, offset = [], 0
        for i in range(0, xs.size(1) - size + stride, stride):
            y, _, att, cnn = self.forward_chunk(xs[:, i: i + size, :], att, cnn, C, L, R, offset)
            outs.append(y[:, :C, :] if i + size < xs.size(1) else y)
            offset += C
        out = torch.cat(outs, dim=1)
        sub = torch.tensor([calc_length(int(t)) for t in lens.tolist()])
        n = int(sub.max()) if sub.numel() else 0   # make_pad_mask's max_len (mask.py:203-226)
        masks = (torch.arange(max(n, 0))[None, :] < sub[:, None]).unsqueeze(1).to(dev)
        return out, masks

    def forward(self, xs, xs_lens, chunk_size: int = 0, left_context_size: int = -1, right_context_size: int = -1,
                **kwargs):
        """encoder.py:461-501 (eval branch)."""
        if chunk_size < 0 or left_context_size < 0 or right_context_size < 0:
            chunk_size, left_context_size, right_context_size = 0, 0, 0
        return self.forward_encoder(xs, xs_lens, chunk_size, left_context_size, right_context_size)

    __call__ = forward

    # ------------------------------------------------------------------ CTC head
    @torch.no_grad()
    def ctc_log_softmax(self, hs: torch.Tensor, want_logp: bool = True, want_ids: bool = True):
        """ctc.py:73-81 log_softmax(ctc_lo(hs)) and its argmax over the vocabulary (int32)."""
        if self.cfg.vocab <= 0:
            raise AssertionError("model has no CTC head")
        shape = hs.shape[:-1]
        enc = hs.reshape(-1, self.cfg.d_model).to(self.device, torch.float32).contiguous()
        rows = enc.shape[0]
        if not want_logp and not want_ids:
            return None, None
        logp = torch.empty(rows, self.cfg.vocab, dtype=torch.float32, device=self.device) if want_logp else None
        ids = torch.empty(rows, dtype=torch.int32, device=self.device) if want_ids else None
        nbytes = self.ctc_ws_bytes(rows, want_logp)
        ws = torch.empty(nbytes, dtype=torch.uint8, device=self.device) if nbytes > 0 else None
        if rows > 0:
            self._ctc_raw(enc, rows, logp, ids, ws)
        return (logp.view(*shape, -1) if logp is not None else None), (ids.view(*shape) if ids is not None else None)

    @torch.no_grad()
    def ctc_collapse(self, ids: torch.Tensor, row_start, row_len, max_silence: Optional[int] = None,
                     blank_id: int = 0):
        """CTC post-processing on device over utterance b = ids[row_start[b] : row_start[b] + row_len[b]].

        max_silence None: remove_duplicates_and_blank (model_utils.py:23-32) -> per utterance
        (tokens, peak frames) lists.  max_silence >= 0: the sentence split of
        get_output_with_timestamps (model_utils.py:174-221) -> per utterance a list of
        (tokens, start_frame, end_frame) segments (80 ms frames).  One kernel launch and one
        device -> host copy of the compacted results."""
        B = len(row_start)
        dev = self.device
        ids = ids.reshape(-1).to(dev, torch.int32).contiguous()
        rows = ids.numel()
        rs = torch.tensor([int(v) for v in row_start], dtype=torch.int32)
        rl = torch.tensor([int(v) for v in row_len], dtype=torch.int32)
        if B and (int((rs + rl).max()) > rows or int(rs.min()) < 0 or int(rl.min()) < 0):
            raise ValueError("utterance row ranges exceed the id tensor")
        seg_mode = max_silence is not None
        ms = int(max_silence) if seg_mode else -1
        if seg_mode and ms < 0:
            raise ValueError("max_silence must be >= 0")
        tok = torch.empty(max(rows, 1), dtype=torch.int32, device=dev)
        tfr = torch.empty(max(rows, 1), dtype=torch.int32, device=dev)
        ntok = torch.zeros(max(B, 1), dtype=torch.int32, device=dev)
        seg = torch.empty(max(rows, 1), 3, dtype=torch.int32, device=dev) if seg_mode else None
        nseg = torch.zeros(max(B, 1), dtype=torch.int32, device=dev) if seg_mode else None
        rs_d, rl_d = rs.to(dev), rl.to(dev)
        _lib.check(_lib.cfm_ctc_collapse(ids.data_ptr(), rs_d.data_ptr(), rl_d.data_ptr(), B, int(blank_id), ms,
                                         tok.data_ptr(), tfr.data_ptr(), ntok.data_ptr(), _lib.ptr(seg),
                                         _lib.ptr(nseg), self._stream()))
        tok_h, tfr_h, ntok_h = tok.cpu().tolist(), tfr.cpu().tolist(), ntok.cpu().tolist()
        out = []
        if not seg_mode:
            for b in range(B):
                s0, n = int(rs[b]), ntok_h[b]
                out.append((tok_h[s0: s0 + n], tfr_h[s0: s0 + n]))
            return out
        seg_h, nseg_h = seg.cpu().tolist(), nseg.cpu().tolist()
        for b in range(B):
            s0, n, ns = int(rs[b]), ntok_h[b], nseg_h[b]
            segs = []
            for k in range(ns):
                t0, start, end = seg_h[s0 + k]
                t1 = seg_h[s0 + k + 1][0] if k + 1 < ns else n
                segs.append((tok_h[s0 + t0: s0 + t1], start, end))
            out.append(segs)
        return out
