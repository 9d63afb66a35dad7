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

from typing import List, Optional

import torch

from . import _lib


class EndlessGraphRunner:
    """Runs the segment schedule of one endless_decode call; middle segments by graph replay."""

    def __init__(self, encoder, C: int, L: int, R: int, trunc: int, seg_len: int, want_out: bool,
                 use_graph: bool = True):
        self.enc = encoder
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

    # ------------------------------------------------------------------ eager step
    def _eager(self, x: torch.Tensor, offset: int):
        enc = self.enc
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

    def _replayable(self, n_frames: int, offset: int) -> bool:
        if not self.use_graph or n_frames != self.seg_len:
            return False
        if self.g_plan is None:   # capture only where the plan no longer depends on offset
            return offset >= max(self.L, 7)
        plan, _, _ = _lib.plan_masked([n_frames], [offset], self.C, self.L, self.R)
        return bool(torch.equal(plan, self.g_plan))

    def step(self, x: torch.Tensor, offset: int, keep_trunc: bool):
        """One segment: returns (CTC ids of the kept rows or None, kept encoder rows or None, kept row
        count).  Rows are kept as chunkformer_model.py:419-431 keeps them: eo[:n], then [:trunc]."""
        if self._replayable(x.shape[0], offset):
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
        out, n = self._eager(x, offset)
        eo = out[:n]
        if keep_trunc:
            eo = eo[: self.trunc]
        ids = None
        if self.vocab > 0 and eo.shape[0] > 0:
            ids = self.enc.ctc_log_softmax(eo, want_logp=False)[1]
        return ids, (eo if self.want_out else None), eo.shape[0]


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

    def __init__(self, encoder, C: int, L: int, R: int, trunc: int, want_out: bool, depth: int = 3):
        if depth < 1:
            raise ValueError(f"pipeline depth {depth} < 1")
        self.enc = encoder
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

    def _buf(self, lst, i, nbytes, dtype, shape=None):
        t = lst[i]
        need = nbytes if shape is None else int(torch.Size(shape).numel())
        if t is None or t.numel() < need:
            lst[i] = torch.empty(need, dtype=dtype, device=self.dev)
        return lst[i]

    def run(self, xs_dev: torch.Tensor, segs):
        """Returns (per-segment CTC ids of the kept rows, per-segment kept encoder rows or None,
        index of the cache pair holding the caches after the last segment); the tensors are ready on
        the caller's current stream."""
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


def stage_slots(num_blocks: int, depth: int):
    """The encoder stages (-1 = front-end, 0 .. num_blocks-1 = layers) cut into `depth` consecutive
    slots [lo, hi] (the longer ones first): EndlessGraphPipeline's stage slots."""
    stages = list(range(-1, num_blocks))
    depth = max(1, min(depth, len(stages)))
    per, extra = divmod(len(stages), depth)
    slots, i = [], 0
    for s in range(depth):
        n = per + (1 if s < extra else 0)
        slots.append((stages[i], stages[i + n - 1]))
        i += n
    return slots


def pipeline_ticks(n_segments: int, depth: int):
    """Tick t of the software pipeline runs slot s of segment t - s for every valid s: a list of
    [(segment, slot), ...] per tick.  Every segment runs its slots 0 .. depth-1 in consecutive ticks,
    and segment k's slot s runs one tick after segment k - 1's (its layer caches) and one tick after
    its own slot s - 1."""
    return [[(t - s, s) for s in range(depth) if 0 <= t - s < n_segments] for t in range(n_segments + depth - 1)]


class EndlessGraphPipeline:
    """endless_decode's segments as a software pipeline of `depth` stage slots whose steady state is
    replayed from HIP graphs (BASELINE configs[3]: context caches carried across graph-captured steps,
    with several segments in flight).

    The encoder stages (-1 = front-end, 0..nb-1 = layers) are cut into `depth` consecutive slots.  Tick
    t runs slot s of segment t - s for every s: those units are independent (segment k's slot s needs
    segment k - 1's slot s, i.e. the layer caches it carries, and its own slot s - 1, both from tick
    t - 1), so within a tick they run on `depth` streams at once, and tick t + 1 starts after tick t.
    A tick whose units all belong to middle segments (the same length and, once offset >= max(L, 7),
    the same plan: streaming.py's module note) is one HIP graph replay; the graph only depends on the
    tick's phase (segment k uses workspace / output slot k % depth and cache pair k % 2), so
    lcm(depth, 2) graphs are captured once per segment geometry.  The first segments (offset 0), the
    ragged last one and the pipeline's fill / drain ticks run the same stage calls eagerly.  Every unit
    is a cfm_encode_masked_stages call with that segment's plan, caches and workspace, so the result is
    bit-identical to the one-call-per-segment loop."""

    def __init__(self, encoder, C: int, L: int, R: int, trunc: int, seg_len: int, want_out: bool, depth: int = 3):
        if depth < 1:
            raise ValueError(f"pipeline depth {depth} < 1")
        self.enc = encoder
        cfg = encoder.cfg
        self.C, self.L, self.R, self.trunc, self.seg_len = C, L, R, trunc, seg_len
        self.want_out = want_out
        dev = encoder.device
        self.dev = dev
        nb, H, dk, d = cfg.num_blocks, cfg.n_heads, cfg.head_dim, cfg.d_model
        self.slots = stage_slots(nb, depth)
        depth = len(self.slots)
        self.depth = depth
        self.att = [torch.zeros(nb, L, H, 2 * dk, device=dev) for _ in range(2)]
        self.cnn = [torch.zeros(nb, d, cfg.conv_lorder, device=dev) for _ in range(2)]
        self.streams = [torch.cuda.Stream(dev) for _ in range(depth)]
        self.ws: List[Optional[torch.Tensor]] = [None] * depth
        self.out: List[Optional[torch.Tensor]] = [None] * depth
        self.ids: List[Optional[torch.Tensor]] = [None] * depth
        self.ctc_ws: List[Optional[torch.Tensor]] = [None] * depth
        self.period = depth if depth % 2 == 0 else 2 * depth
        self.graphs: dict = {}
        self.g_plan = None
        self.g_feats = torch.zeros(max(seg_len, 1), cfg.input_dim, device=dev)
        self.vocab = cfg.vocab
        self.replayed = 0   # ticks replayed from graphs in the last run (tests / bench)

    def _buf(self, lst, i, n, dtype) -> None:
        t = lst[i]
        if t is None or t.numel() < n:
            lst[i] = torch.empty(n, dtype=dtype, device=self.dev)
            self.graphs.clear()   # captured graphs hold the old buffer's address

    def _unit(self, seg: dict, slot: int, st) -> None:
        """Slot `slot`'s stage calls for one segment on stream `st` (+ the CTC head after the last)."""
        enc = self.enc
        k, p = seg["k"], seg["k"] % self.depth
        c = k % 2
        lo, hi = self.slots[slot]
        _lib.check(_lib.cfm_encode_masked_stages(
            enc._h, seg["feats"].data_ptr(), seg["plan"].data_ptr(), seg["plan_dev"].data_ptr(),
            self.att[c].data_ptr(), self.cnn[c].data_ptr(), int(self.trunc), self.att[1 - c].data_ptr(),
            self.cnn[1 - c].data_ptr(), self.out[p].data_ptr(), self.ws[p].data_ptr(), seg["wsb"], lo, hi,
            st.cuda_stream))
        if slot == self.depth - 1 and self.vocab > 0 and seg["rows"] > 0:
            with torch.cuda.stream(st):
                enc._ctc_raw(self.out[p], seg["rows"], None, self.ids[p], self.ctc_ws[p])

    def _tick(self, units, graph_key=None) -> None:
        """One tick: its units on `depth` streams (fork from / join into the caller's stream), either
        eagerly or by replaying (capturing first) the graph of `graph_key`."""
        caller = torch.cuda.current_stream(self.dev)
        if graph_key is not None:
            g = self.graphs.get(graph_key)
            if g is None:
                g = torch.cuda.CUDAGraph()
                cap = self.streams[0]
                cap.wait_stream(caller)
                with torch.cuda.graph(g, stream=cap):
                    self._fork_join(units, cap)
                self.graphs[graph_key] = g
            g.replay()
            self.replayed += 1
            return
        self._fork_join(units, caller)

    def _fork_join(self, units, base) -> None:
        for i, (seg, slot) in enumerate(units):
            st = self.streams[i]
            if st is not base:
                st.wait_stream(base)
            self._unit(seg, slot, st)
        for i in range(len(units)):
            if self.streams[i] is not base:
                base.wait_stream(self.streams[i])

    def run(self, xs_dev: torch.Tensor, segs):
        """Returns (per-segment CTC ids of the kept rows, per-segment kept encoder rows or None, index of
        the cache pair holding the caches after the last segment), ready on the caller's stream."""
        enc, C, L, R, D = self.enc, self.C, self.L, self.R, self.depth
        d = enc.cfg.d_model
        self.att[0].zero_()
        self.cnn[0].zero_()
        self.replayed = 0
        caller = torch.cuda.current_stream(self.dev)
        n = len(segs)
        if n == 0:
            return [], [], 0
        info, offset = [], 0
        for k, (start, stop, keep_trunc, _) in enumerate(segs):
            n_frames = stop - start
            plan, n_chunks, out_lens = _lib.plan_masked([n_frames], [offset], C, L, R)
            N = n_chunks[0]
            kept = min(out_lens[0], self.trunc) if keep_trunc else out_lens[0]
            info.append({"k": k, "x": xs_dev[start:stop], "plan": plan, "N": N, "n": out_lens[0], "rows": kept,
                         "wsb": int(_lib.cfm_workspace_bytes_masked(enc._h, N, C, L, R)), "len": n_frames})
            offset += kept
        # the graph plan: the first middle segment whose plan no longer depends on the offset
        if self.g_plan is None:
            for s in info:
                if s["len"] == self.seg_len and sum(s2["rows"] for s2 in info[: s["k"]]) >= max(L, 7):
                    self.g_plan = s["plan"]
                    self.g_plan_dev = enc._upload(s["plan"])
                    break
        for s in info:
            s["graph"] = self.g_plan is not None and s["len"] == self.seg_len and torch.equal(s["plan"], self.g_plan)
            if s["graph"]:
                s["plan"], s["plan_dev"], s["feats"] = self.g_plan, self.g_plan_dev, self.g_feats
            else:
                s["plan_dev"] = enc._upload(s["plan"])
                s["feats"] = s["x"].contiguous()
        max_rows = max([s["rows"] for s in info] + [1])
        ctc_b = enc.ctc_ws_bytes(max_rows, False) if self.vocab > 0 else 0   # 0 on the fused argmax head
        for p in range(D):   # slot buffers sized for the largest segment
            self._buf(self.ws, p, max(s["wsb"] for s in info), torch.uint8)
            self._buf(self.out, p, max(s["N"] for s in info) * C * d, torch.float32)
            self._buf(self.ids, p, max_rows, torch.int32)
            if ctc_b > 0:
                self._buf(self.ctc_ws, p, ctc_b, torch.uint8)
        ids_out: List[Optional[torch.Tensor]] = [None] * n
        eo_out: List[Optional[torch.Tensor]] = [None] * n
        for t, tick in enumerate(pipeline_ticks(n, D)):
            units = [(info[k], s) for k, s in tick]
            full = len(units) == D and all(u[0]["graph"] for u in units)
            if units and units[0][1] == 0 and units[0][0]["graph"]:
                self.g_feats[: units[0][0]["len"]].copy_(units[0][0]["x"])   # the graph's input rows
            self._tick(units, (t % self.period) if full else None)
            done = t - (D - 1)   # the segment whose last slot ran in this tick
            if 0 <= done < n:
                s = info[done]
                p = done % D
                eo = self.out[p][: s["N"] * C * d].view(s["N"] * C, d)[: s["rows"]]
                if self.vocab > 0 and s["rows"] > 0:
                    ids_out[done] = self.ids[p][: s["rows"]].clone()
                if self.want_out:
                    eo_out[done] = eo.clone()
        self._keep = info
        return ids_out, eo_out, n % 2
