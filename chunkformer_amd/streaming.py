"""HIP-graph replay of endless_decode's segment steps (BASELINE configs[3]).

The reference's endless_decode (chunkformer_model.py:321-459) calls
forward_parallel_chunk once per segment of one long utterance, carrying the attention
/ conv caches (attention.py:466-467, convolution.py:228-230) and `offset` from one
segment to the next, then runs the CTC head on the kept rows (436-438).

Every segment between the first and the last has the same input length
(step + 7 + rel_right fbank frames) and, once `offset` >= max(L, 7), the same plan:
the packer's masks only look at `offset` through max(0, L - offset - 64c) and
max(0, 7 - offset - 64c) (encoder.py:625-645, planner.cpp).  So one segment step --
front-end, 12 blocks with caches in/out, after_norm, CTC argmax of the kept rows --
is captured once into a HIP graph (torch.cuda.CUDAGraph over libcfm's stream-ordered,
allocation-free C-ABI calls) and replayed for every middle segment.  The caches
ping-pong between two fixed buffer pairs, so two graphs are captured (A -> B and
B -> A).  The first segment (offset 0) and the ragged last segment run eagerly through
the same entry points; each replayed segment's plan is re-derived on the host and
compared with the captured one, so a plan mismatch falls back to the eager call
instead of replaying the wrong masks.
"""
from __future__ import annotations

from collections import OrderedDict
from typing import List, Optional

import torch

from . import _lib

def destroy_graphs(entries, device) -> None:
    """Destroy captured graphs (CUDAGraph objects, or (graph, events) tuples): the device is synchronised
    first, so no replay of them is still in flight when hipGraphExecDestroy runs, then each graph is reset
    before the events recorded during its capture (kept beside it) are released."""
    entries = [e for e in entries if e is not None]
    if not entries:
        return
    torch.cuda.synchronize(device)
    for e in entries:
        (e[0] if isinstance(e, tuple) else e).reset()


class EndlessGraphRunner:
    """Runs the segment schedule of one endless_decode call; middle segments by graph replay."""

    def __init__(self, encoder, C: int, L: int, R: int, trunc: int, seg_len: int, want_out: bool,
                 use_graph: bool = True, trim: bool = False):
        self.enc = encoder
        self.trim = trim   # truncated segments skip the rows past trunc (model option "trim_right")
        cfg = encoder.cfg
        self.C, self.L, self.R, self.trunc = C, L, R, trunc
        self.seg_len = seg_len
        self.want_out = want_out
        self.use_graph = use_graph
        dev = encoder.device
        self.dev = dev
        nb, H, dk, d = cfg.num_blocks, cfg.n_heads, cfg.head_dim, cfg.d_model
        # caches: pair 0 and pair 1 (ping-pong across graph replays)
        self.att = [torch.zeros(nb, L, H, 2 * dk, device=dev) for _ in range(2)]
        self.cnn = [torch.zeros(nb, d, cfg.conv_lorder, device=dev) for _ in range(2)]
        self.cur = 0   # index of the pair holding the carried caches
        self.graphs: List[Optional[torch.cuda.CUDAGraph]] = [None, None]
        self.g_plan = None
        self.vocab = cfg.vocab

    def reset(self) -> None:
        """Start a new utterance: zero caches (chunkformer_model.py:376-379); graphs are kept."""
        self.cur = 0
        self.att[0].zero_()
        self.cnn[0].zero_()

    def close(self) -> None:
        """Destroy the captured graphs (the runner is being replaced); the buffers go with the runner."""
        destroy_graphs(self.graphs, self.dev)
        self.graphs = [None, None]
        self.g_plan = None

    # ------------------------------------------------------------------ eager step
    def _eager(self, x: torch.Tensor, offset: int, keep_trunc: bool):
        enc = self.enc
        enc._set_trim(self.trim and keep_trunc)
        n_frames = x.shape[0]
        plan, n_chunks, out_lens = _lib.plan_masked([n_frames], [offset], self.C, self.L, self.R)
        N = n_chunks[0]
        plan_dev = enc._upload(plan)
        out = torch.empty(N * self.C, enc.cfg.d_model, device=self.dev)
        ws = enc._workspace(_lib.cfm_workspace_bytes_masked(enc._h, N, self.C, self.L, self.R))
        src, dst = self.cur, 1 - self.cur
        enc._encode_masked_raw(x.contiguous(), plan, plan_dev, self.att[src], self.cnn[src], self.trunc,
                               self.att[dst], self.cnn[dst], out, ws)
        self.cur = dst
        self._keep = (plan, plan_dev)
        return out, out_lens[0]

    # ------------------------------------------------------------------ graph step
    def _capture(self, offset: int):
        enc = self.enc
        plan, n_chunks, out_lens = _lib.plan_masked([self.seg_len], [offset], self.C, self.L, self.R)
        N = n_chunks[0]
        self.g_plan = plan
        self.g_plan_dev = enc._upload(plan)
        self.g_n = out_lens[0]
        self.g_rows = min(self.g_n, self.trunc)
        self.g_feats = torch.zeros(self.seg_len, enc.cfg.input_dim, device=self.dev)
        self.g_out = torch.empty(N * self.C, enc.cfg.d_model, device=self.dev)
        self.g_ws = torch.empty(_lib.cfm_workspace_bytes_masked(enc._h, N, self.C, self.L, self.R),
                                dtype=torch.uint8, device=self.dev)
        if self.vocab > 0:
            self.g_ids = torch.empty(self.g_rows, dtype=torch.int32, device=self.dev)
            nb = enc.ctc_ws_bytes(self.g_rows, False)   # 0 on the fused argmax head
            self.g_ctc_ws = torch.empty(nb, dtype=torch.uint8, device=self.dev) if nb > 0 else None
        torch.cuda.current_stream(self.dev).synchronize()
        self.enc._set_trim(self.trim)   # only truncated middle segments replay (_replayable)

        def body(src: int):
            dst = 1 - src
            enc._encode_masked_raw(self.g_feats, self.g_plan, self.g_plan_dev, self.att[src], self.cnn[src],
                                   self.trunc, self.att[dst], self.cnn[dst], self.g_out, self.g_ws)
            if self.vocab > 0:
                enc._ctc_raw(self.g_out, self.g_rows, None, self.g_ids, self.g_ctc_ws)

        # warm the launch path on a side stream (libcfm's one-time queries happen outside capture),
        # on scratch caches so the carried state is untouched
        saved = [(a.clone(), c.clone()) for a, c in zip(self.att, self.cnn)]
        side = torch.cuda.Stream(self.dev)
        self._capture_stream = side   # kept alive with the graphs captured on it
        side.wait_stream(torch.cuda.current_stream(self.dev))
        with torch.cuda.stream(side):
            body(0)
        torch.cuda.current_stream(self.dev).wait_stream(side)
        for src in (0, 1):
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g, stream=side):
                body(src)
            self.graphs[src] = g
        for (a, c), (sa, sc) in zip(zip(self.att, self.cnn), saved):
            a.copy_(sa)
            c.copy_(sc)

    def _replayable(self, n_frames: int, offset: int, keep_trunc: bool) -> bool:
        if not self.use_graph or n_frames != self.seg_len or not keep_trunc:
            return False
        if self.g_plan is None:   # capture only where the plan no longer depends on offset
            return offset >= max(self.L, 7)
        plan, _, _ = _lib.plan_masked([n_frames], [offset], self.C, self.L, self.R)
        return bool(torch.equal(plan, self.g_plan))

    def step(self, x: torch.Tensor, offset: int, keep_trunc: bool):
        """One segment: returns (CTC ids of the kept rows or None, kept encoder rows or None, kept row
        count).  Rows are kept as chunkformer_model.py:419-431 keeps them: eo[:n], then [:trunc]."""
        if self._replayable(x.shape[0], offset, keep_trunc):
            if self.graphs[0] is None:
                self._capture(offset)
            self.g_feats.copy_(x)
            self.graphs[self.cur].replay()
            self.cur = 1 - self.cur
            eo = self.g_out[: self.g_n]
            if keep_trunc:
                eo = eo[: self.trunc]
            if eo.shape[0] == self.g_rows and self.vocab > 0:
                ids = self.g_ids.clone()
            else:
                ids = self.enc.ctc_log_softmax(eo, want_logp=False)[1] if self.vocab > 0 else None
            return ids, (eo.clone() if self.want_out else None), eo.shape[0]
        out, n = self._eager(x, offset, keep_trunc)
        eo = out[:n]
        if keep_trunc:
            eo = eo[: self.trunc]
        ids = None
        if self.vocab > 0 and eo.shape[0] > 0:
            ids = self.enc.ctc_log_softmax(eo, want_logp=False)[1]
        return ids, (eo if self.want_out else None), eo.shape[0]


# Launch parameters while several segments are in flight (each launch then shares the chip with the
# other streams' kernels): the K = 512 weight-stationary GEMMs of a segment (< 32k rows) on a quarter
# of the CUs (each workgroup then takes 4x the row tiles per weight-tile fill), ring attention runs of
# >= 16 chunks per workgroup.  tbd 1800, 16 h (same box): graph pipeline 22.2 -> 23.9 M frames/s, eager
# pipeline 22.2 -> 23.3 M; tbd 7200 segments (45k rows) are not affected.
PIPELINE_OPTS = {"wsp_small_div": 4, "attn_min_chunks": 16}


class EndlessPipeline:
    """endless_decode's segments with `depth` in flight (MI355X streams, no graph): segment k runs on
    stream k % depth and its encoder layer l waits only for segment k - 1's layer l (the attention /
    conv caches it carries, attention.py:466-467, convolution.py:228-230), so segment k + 1's
    front-end and early layers overlap segment k's later layers.  At the reference's default
    total_batch_duration (1800 s: 12.7k-row segments) single launches leave most CUs idle in their
    tail rounds; the next segments' kernels fill them (depth 3 measured best: 20.5M frames/s at
    tbd 1800 vs 18.8M at depth 2, 18.5M at depth 4 and 14.9M for the graph-replayed sequential loop).  Each stage is a cfm_encode_masked_stages
    call (stage -1: front-end + relative positions; stage l: layer l), so the result is bit-identical
    to the one-call-per-segment loop (same kernels, same inputs, same order per segment)."""

    def __init__(self, encoder, C: int, L: int, R: int, trunc: int, want_out: bool, depth: int = 3,
                 trim: bool = False):
        if depth < 1:
            raise ValueError(f"pipeline depth {depth} < 1")
        self.enc = encoder
        self.trim = trim
        self.depth = depth
        cfg = encoder.cfg
        self.C, self.L, self.R, self.trunc = C, L, R, trunc
        self.want_out = want_out
        dev = encoder.device
        self.dev = dev
        nb, H, dk, d = cfg.num_blocks, cfg.n_heads, cfg.head_dim, cfg.d_model
        self.att = [torch.zeros(nb, L, H, 2 * dk, device=dev) for _ in range(2)]
        self.cnn = [torch.zeros(nb, d, cfg.conv_lorder, device=dev) for _ in range(2)]
        # segment k: stream / workspace / output k % depth; caches pair k % 2 in, (k + 1) % 2 out (two
        # pairs suffice at any depth: layer l of segment k + 1 starts after layer l of segment k)
        self.streams = [torch.cuda.Stream(dev) for _ in range(depth)]
        self.ws: List[Optional[torch.Tensor]] = [None] * depth
        self.out: List[Optional[torch.Tensor]] = [None] * depth

    def close(self) -> None:
        """Nothing captured: the streams' last work is joined so the buffers can go."""
        torch.cuda.synchronize(self.dev)

    def _buf(self, lst, i, nbytes, dtype, shape=None):
        t = lst[i]
        need = nbytes if shape is None else int(torch.Size(shape).numel())
        if t is None or t.numel() < need:
            lst[i] = torch.empty(need, dtype=dtype, device=self.dev)
        return lst[i]

    def run(self, xs_dev: torch.Tensor, segs):
        """Returns (per-segment CTC ids of the kept rows, per-segment kept encoder rows or None,
        index of the cache pair holding the caches after the last segment); the tensors are ready on
        the caller's current stream.  Launch parameters for segments in flight: PIPELINE_OPTS."""
        with self.enc.scoped_options(**PIPELINE_OPTS):
            try:
                return self._run(xs_dev, segs)
            finally:
                self.enc._set_trim(False)

    def _run(self, xs_dev: torch.Tensor, segs):
        enc, C, L, R = self.enc, self.C, self.L, self.R
        nb, d = enc.cfg.num_blocks, enc.cfg.d_model
        self.att[0].zero_()
        self.cnn[0].zero_()
        caller = torch.cuda.current_stream(self.dev)
        for s in self.streams:
            s.wait_stream(caller)   # inputs and the zeroed caches
        ids_out, eo_out, keep = [], [], []
        prev = None
        offset = 0
        for k, (start, stop, keep_trunc, _) in enumerate(segs):
            p = k % self.depth
            c = k % 2
            st = self.streams[p]
            x = xs_dev[start:stop]
            n_frames = stop - start
            plan, n_chunks, out_lens = _lib.plan_masked([n_frames], [offset], C, L, R)
            N = n_chunks[0]
            wsb = int(_lib.cfm_workspace_bytes_masked(enc._h, N, C, L, R))
            cur = []
            enc._set_trim(self.trim and keep_trunc)
            with torch.cuda.stream(st):
                plan_dev = plan.pin_memory().to(self.dev, non_blocking=True)
                ws = self._buf(self.ws, p, wsb, torch.uint8)
                out = self._buf(self.out, p, None, torch.float32, (N * C, d))
                src, dst = self.att[c], self.att[1 - c]
                csrc, cdst = self.cnn[c], self.cnn[1 - c]
                for stage in range(-1, nb):
                    if stage >= 0 and prev is not None:
                        st.wait_event(prev[stage])
                    _lib.check(_lib.cfm_encode_masked_stages(
                        enc._h, x.data_ptr(), plan.data_ptr(), plan_dev.data_ptr(), src.data_ptr(), csrc.data_ptr(),
                        int(self.trunc), dst.data_ptr(), cdst.data_ptr(), out.data_ptr(), ws.data_ptr(), wsb,
                        stage, stage, st.cuda_stream))
                    if stage >= 0:
                        ev = torch.cuda.Event()
                        ev.record(st)
                        cur.append(ev)
                n = out_lens[0]
                eo = out[: N * C * d].view(N * C, d)[:n]
                if keep_trunc:
                    eo = eo[: self.trunc]
                ids = enc.ctc_log_softmax(eo, want_logp=False)[1] if enc.cfg.vocab > 0 and eo.shape[0] else None
                eo_c = eo.clone() if self.want_out else None
                for t in (ids, eo_c):
                    if t is not None:
                        t.record_stream(caller)
                ids_out.append(ids)
                eo_out.append(eo_c)
            keep.append((plan, plan_dev))
            offset += eo.shape[0]
            prev = cur
        for s in self.streams:
            caller.wait_stream(s)
        self._keep = keep
        return ids_out, eo_out, len(segs) % 2


def graph_blocks(n: int, block: int, period: int):
    """EndlessGraphPipeline's schedule (host logic): the n segments as [(start, count, phase), ...] in
    order -- consecutive blocks of at most `block` segments, each replayed from one captured graph; a
    block's graph depends on its first segment's phase start % period (stream, workspace and cache
    slots cycle with that period) and on its segments' plans."""
    return [(k0, min(block, n - k0), k0 % period) for k0 in range(0, n, max(1, block))]


class EndlessGraphPipeline:
    """endless_decode's segments with `depth` in flight (as EndlessPipeline: segment k on stream
    k % depth, its layer l waiting only for segment k - 1's layer l), all of them replayed from HIP
    graphs (BASELINE configs[3]: context caches carried across graph-captured steps,
    several segments in flight).

    Every segment runs from HIP graphs: a block of up to `block` (128: a 16 h input at tbd 1800, 65
    segments, is one block) consecutive segments is captured once as ONE graph holding the whole
    multi-stream pipeline of those segments -- every stage call, the per-layer cross-stream event
    edges, the CTC head and the copies of each segment's kept rows / ids into the block's output
    slots.  Segment k uses stream, workspace and output slot k % depth and cache pair k % 2, so a
    block's graph is keyed by its first segment's phase k mod lcm(depth, 2) and by its segments'
    plans (the offset-0 first segment and the ragged last one have their own; the middle ones, once
    offset >= max(L, 7), share one: streaming.py's module note), lengths and kept rows; the device
    plans are kept per distinct plan, so a repeated input (or the middle blocks of any input) replays
    without re-capture.  Inside a replay the segments overlap exactly as in the eager pipeline, with
    no drain between the first, middle and last segments; a block's first segment starts after the
    previous block (one drain per block).  The calls are the ones the eager pipeline makes, so the
    result is bit-identical to the one-call-per-segment loop.  With `fe_reuse` a segment's first
    front-end windows -- the previous segment's last complete ones, the same frames -- are copied from
    a carry buffer the previous segment's stage -1 filled (native fe_carry), not recomputed."""

    # captured block graphs kept per runner (least recently replayed destroyed first): a service decoding
    # inputs of many lengths holds at most this many, each with its events and no allocations
    MAX_GRAPHS = 8

    def __init__(self, encoder, C: int, L: int, R: int, trunc: int, seg_len: int, want_out: bool, depth: int = 3,
                 block: int = 128, trim: bool = False, fe_reuse: bool = False, max_graphs: int = MAX_GRAPHS):
        if depth < 1:
            raise ValueError(f"pipeline depth {depth} < 1")
        self.enc = encoder
        self.trim = trim
        # the next segment's first front-end windows are this segment's last complete ones (same frames):
        # their output rows are carried in self.carry instead of recomputed (native "fe_carry")
        self.fe_reuse = fe_reuse
        self.carry: Optional[torch.Tensor] = None
        cfg = encoder.cfg
        self.C, self.L, self.R, self.trunc, self.seg_len = C, L, R, trunc, seg_len
        self.want_out = want_out
        dev = encoder.device
        self.dev = dev
        nb, H, dk, d = cfg.num_blocks, cfg.n_heads, cfg.head_dim, cfg.d_model
        self.depth = depth
        self.period = depth if depth % 2 == 0 else 2 * depth
        self.block = max(1, block)
        self.att = [torch.zeros(nb, L, H, 2 * dk, device=dev) for _ in range(2)]
        self.cnn = [torch.zeros(nb, d, cfg.conv_lorder, device=dev) for _ in range(2)]
        self.streams = [torch.cuda.Stream(dev) for _ in range(depth)]
        self.ws: List[Optional[torch.Tensor]] = [None] * depth
        self.out: List[Optional[torch.Tensor]] = [None] * depth
        self.ctc_ws: List[Optional[torch.Tensor]] = [None] * depth
        # the graphs' fixed input / output slots, by position in a block
        self.g_feats: List[Optional[torch.Tensor]] = [None] * self.block
        self.g_ids: List[Optional[torch.Tensor]] = [None] * self.block
        self.g_eo: List[Optional[torch.Tensor]] = [None] * self.block
        # block key -> (graph, events recorded in its capture), least recently replayed first
        self.graphs: "OrderedDict[tuple, tuple]" = OrderedDict()
        self.max_graphs = max(1, int(max_graphs))
        self.plans: dict = {}   # plan bytes -> (host plan, device plan, id): the graphs' plan inputs
        self._next_pid = 0
        self.vocab = cfg.vocab
        self.replayed = 0   # segments replayed from graphs in the last run (tests / bench)
        self.captures = 0   # graphs captured over the runner's life (tests)

    def close(self) -> None:
        """Destroy every captured graph (runner replaced, or a buffer the graphs point at reallocated)."""
        destroy_graphs(list(self.graphs.values()), self.dev)
        self.graphs.clear()

    def _buf(self, lst, i, n, dtype) -> torch.Tensor:
        t = lst[i]
        if t is None or t.numel() < n:
            self.close()   # the captured graphs hold the old buffer's address (and may still run on it)
            lst[i] = None
            lst[i] = torch.empty(n, dtype=dtype, device=self.dev)
        return lst[i]

    def _segment(self, seg: dict, prev, ids_dst, eo_dst):
        """Segment seg["k"]'s stage calls on stream k % depth, layer l after `prev[l]` (the previous
        segment's layer-l event); its CTC ids into ids_dst and (want_out) its kept rows into eo_dst.
        Returns its per-layer events."""
        enc, C = self.enc, self.C
        d = enc.cfg.d_model
        k = seg["k"]
        p, c = k % self.depth, k % 2
        st = self.streams[p]
        cur = []
        enc._set_trim(self.trim and seg["keep"])
        if self.fe_reuse:
            enc._set_fe_carry(self.carry.data_ptr() if self.carry is not None else 0, seg["reuse"], seg["save_from"])
        for stage in range(-1, enc.cfg.num_blocks):
            if stage == -1 and seg["reuse"] > 0 and prev is not None:
                st.wait_event(prev[-1])   # the previous segment's front-end filled the carry
            if stage >= 0 and prev is not None:
                st.wait_event(prev[stage])
            _lib.check(_lib.cfm_encode_masked_stages(
                enc._h, seg["feats"].data_ptr(), seg["plan"].data_ptr(), seg["plan_dev"].data_ptr(),
                self.att[c].data_ptr(), self.cnn[c].data_ptr(), int(self.trunc), self.att[1 - c].data_ptr(),
                self.cnn[1 - c].data_ptr(), self.out[p].data_ptr(), self.ws[p].data_ptr(), seg["wsb"], stage, stage,
                st.cuda_stream))
            if stage >= 0 or self.fe_reuse:   # (the front-end's event last: prev[-1])
                ev = torch.cuda.Event()
                ev.record(st)
                cur.append(ev)
        if self.fe_reuse:
            cur.append(cur.pop(0))
        rows = seg["rows"]
        if rows > 0:
            with torch.cuda.stream(st):
                eo = self.out[p][: seg["N"] * C * d].view(seg["N"] * C, d)[:rows]
                if ids_dst is not None:
                    enc._ctc_raw(eo, rows, None, ids_dst, self.ctc_ws[p])
                if eo_dst is not None:
                    eo_dst.copy_(eo)
        return cur

    def run(self, xs_dev: torch.Tensor, segs):
        """Returns (per-segment CTC ids of the kept rows, per-segment kept encoder rows or None, index of
        the cache pair holding the caches after the last segment), ready on the caller's stream.
        Launch parameters for segments in flight: PIPELINE_OPTS (baked into the captured graphs)."""
        with self.enc.scoped_options(**PIPELINE_OPTS):
            try:
                return self._run(xs_dev, segs)
            finally:
                self.enc._set_trim(False)
                if self.fe_reuse:
                    self.enc._set_fe_carry(0, 0, -1)

    def _run(self, xs_dev: torch.Tensor, segs):
        enc, C, L, R, D = self.enc, self.C, self.L, self.R, self.depth
        d = enc.cfg.d_model
        self.replayed = 0
        caller = torch.cuda.current_stream(self.dev)
        n = len(segs)
        if n == 0:
            return [], [], 0
        self.att[0].zero_()
        self.cnn[0].zero_()
        info, offset = [], 0
        for k, (start, stop, keep_trunc, _) in enumerate(segs):
            n_frames = stop - start
            plan, n_chunks, out_lens = _lib.plan_masked([n_frames], [offset], C, L, R)
            N = n_chunks[0]
            # rows of out[:n] with Python slice semantics, as the reference's encoder_out[:, :encoder_len]
            # (chunkformer_model.py:419): a segment of < 15 frames has calc_length -1, which drops the
            # last row of its one padded chunk instead of returning none (EndlessPipeline: eo[:n])
            n_rows = len(range(N * C)[: out_lens[0]])
            kept = min(n_rows, self.trunc) if keep_trunc else n_rows
            info.append({"k": k, "x": xs_dev[start:stop], "plan": plan, "N": N, "rows": kept, "keep": keep_trunc,
                         "wsb": int(_lib.cfm_workspace_bytes_masked(enc._h, N, C, L, R)), "len": n_frames,
                         "start": start, "reuse": 0, "save_from": -1})
            offset += kept
        if self.fe_reuse:
            for a, b in zip(info, info[1:]):
                # segment b starts trunc rows (8 trunc frames) after a: a's windows trunc / C .. are b's first
                # ones; only windows a holds whole (8C + 7 frames inside a) are carried
                if not a["keep"] or self.trunc % C or b["start"] - a["start"] != 8 * self.trunc:
                    continue
                complete = min(a["N"], max(0, (a["len"] - 8 * C - 7) // (8 * C) + 1))
                n_c = min(complete - self.trunc // C, b["N"])
                if n_c > 0:
                    a["save_from"], b["reuse"] = self.trunc // C, n_c
            need = max([(s_["N"] - s_["save_from"]) * C * d for s_ in info if s_["save_from"] >= 0] + [0])
            if need and (self.carry is None or self.carry.numel() < need):
                self.close()   # the captured graphs hold the old carry's address
                self.carry = None
                self.carry = torch.empty(need, dtype=torch.float32, device=self.dev)
        # every segment runs from a captured graph: device plans are kept per distinct plan (the middle
        # segments share one; the first, offset-0 segment and the ragged last one have their own), and a
        # block's graph is keyed by its phase and its segments' plans / lengths / kept rows, so the middle
        # blocks of any input and the whole of a same-length input replay without re-capture
        for s in info:
            pk = s["plan"].numpy().tobytes()
            ent = self.plans.get(pk)
            if ent is None:
                ent = (s["plan"], enc._upload(s["plan"]), self._next_pid)
                self._next_pid += 1
                self.plans[pk] = ent
            s["plan"], s["plan_dev"], s["pid"] = ent
        max_rows = max([s["rows"] for s in info] + [1])
        ctc_b = enc.ctc_ws_bytes(max_rows, False) if self.vocab > 0 else 0   # 0 on the fused argmax head
        for p in range(D):   # slot buffers sized for the largest segment
            self._buf(self.ws, p, max(s["wsb"] for s in info), torch.uint8)
            self._buf(self.out, p, max(s["N"] for s in info) * C * d, torch.float32)
            if ctc_b > 0:
                self._buf(self.ctc_ws, p, ctc_b, torch.uint8)
        nblk = min(self.block, n)
        for i in range(nblk):
            self._buf(self.g_feats, i, self.seg_len * enc.cfg.input_dim, torch.float32)
            if self.vocab > 0:
                self._buf(self.g_ids, i, max_rows, torch.int32)
            if self.want_out:
                self._buf(self.g_eo, i, max_rows * d, torch.float32)
        ids_out: List[Optional[torch.Tensor]] = [None] * n
        eo_out: List[Optional[torch.Tensor]] = [None] * n
        for k0, cnt, phase in graph_blocks(n, self.block, self.period):
            # a block starts after everything before it (inputs, zeroed caches, the previous block)
            for st in self.streams:
                caller.wait_stream(st)
            for i in range(cnt):
                s = info[k0 + i]
                self.g_feats[i][: s["len"] * enc.cfg.input_dim].view(s["len"], -1).copy_(s["x"])
            key = (phase, tuple((s["pid"], s["len"], s["rows"], s["keep"], s["reuse"], s["save_from"])
                                for s in info[k0: k0 + cnt]))
            entry = self.graphs.get(key)
            if entry is None and len(self.graphs) >= self.max_graphs:
                # the least recently replayed graph goes (after a device sync: it may still be running)
                destroy_graphs([self.graphs.popitem(last=False)[1]], self.dev)
            if entry is None:
                g = torch.cuda.CUDAGraph()
                cap = self.streams[0]
                cap.wait_stream(caller)
                # every event recorded inside the capture (the per-layer edges between the streams and the
                # fork / join) is kept with the graph, which can refer to them
                keep: List[torch.cuda.Event] = []

                def edge(dst, src):
                    e = torch.cuda.Event()
                    e.record(src)
                    dst.wait_event(e)
                    keep.append(e)

                with torch.cuda.graph(g, stream=cap):
                    for st in self.streams[1:]:
                        edge(st, cap)
                    gp = None
                    for i in range(cnt):
                        s = dict(info[k0 + i])
                        s["feats"] = self.g_feats[i]
                        gp = self._segment(s, gp,
                                           self.g_ids[i][: s["rows"]] if self.vocab > 0 else None,
                                           self.g_eo[i][: s["rows"] * d].view(s["rows"], d) if self.want_out else None)
                        keep.extend(gp)
                    for st in self.streams[1:]:
                        edge(cap, st)
                entry = (g, keep)
                self.graphs[key] = entry
                self.captures += 1
                caller.wait_stream(cap)
            self.graphs.move_to_end(key)
            entry[0].replay()
            self.replayed += cnt
            for i in range(cnt):
                rows = info[k0 + i]["rows"]
                if self.vocab > 0 and rows > 0:
                    ids_out[k0 + i] = self.g_ids[i][:rows].clone()
                if self.want_out:
                    eo_out[k0 + i] = self.g_eo[i][: rows * d].view(rows, d).clone()
            for st in self.streams:
                st.wait_stream(caller)
        for st in self.streams:
            caller.wait_stream(st)
        self._keep = info
        # device plans no live graph and no segment of this run refers to are released
        live = {p for key in self.graphs for p, *_ in key[1]} | {s["pid"] for s in info}
        for pk in [pk for pk, ent in self.plans.items() if ent[2] not in live]:
            del self.plans[pk]
        return ids_out, eo_out, n % 2
