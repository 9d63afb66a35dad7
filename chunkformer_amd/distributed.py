"""Multi-GPU masked-batch scheduling: one process per GPU, torch.distributed over RCCL.

The reference has no inference-time distribution; this is the build's own
component.  Utterances of a masked batch are independent (batch-composition invariance,
SURVEY §A.1), so the packed chunk stream is cut with NO exchange during the encoder:

  plan_shards    the work units ("pieces") of every rank: whole utterances placed by LPT
                 bin-packing of chunk counts, and -- for an utterance longer than a rank's share
                 of the batch -- contiguous segments of it on the utterance's own chunk grid with
                 a recomputed halo on both sides, cut to fill every rank to one common level.
                 The plan is a pure function of the lengths, so every rank derives every other
                 rank's row counts without communicating.
  run_pieces     one forward_parallel_chunk call over a rank's pieces (+ the fused CTC head),
                 returning the kept rows
  gather_ids     the one collective: all_gather_into_tensor of every rank's kept CTC ids
                 (int32, padded to the largest rank), reassembled per utterance on every rank
  gather_logp    the same for bf16 CTC log-probs ([rows, V] per rank)

Halo: an encoder layer reaches ceil(L/C) chunks through attention and, through the conv
module's 7-frame context, ceil(7/C) more chunks of attention outputs, so 12 layers at
C=64, L=R=128 see 3 x 12 = 36 chunks per side.  Kept chunks at least that far
from a cut compute from bit-identical inputs at every layer, so they equal the unsharded run.
The reference's own endless_decode uses a right context of r + max(C, r)(nb-1) frames (24
chunks, chunkformer_model.py:344-371); `halo` can be set lower (to 24) to mirror it.
"""
from __future__ import annotations

import heapq
import math
from dataclasses import dataclass
from typing import Dict, List, Optional, Sequence, Tuple

import numpy as np
import torch
import torch.distributed as dist


def chunks_of(T: int, C: int) -> int:
    """n_chunk of one utterance (encoder.py:556-562)."""
    size, step = (C - 1) * 8 + 15, 8 * C
    n_pad = (step - ((T - size) % step)) % step if T >= size else size - T
    return (T + n_pad - size) // step + 1


def out_len(T: int) -> int:
    """calc_length (subsampling.py:270-288): subsampled frames of T fbank frames."""
    return max(0, 1 + (int(T) - 15) // 8)


def receptive_halo(C: int, L: int, R: int, num_blocks: int, kernel_size: int = 15) -> Tuple[int, int]:
    """Chunks per side a kept chunk depends on after `num_blocks` layers (left, right)."""
    conv = math.ceil((kernel_size // 2) / C)
    return num_blocks * (math.ceil(L / C) + conv), num_blocks * (math.ceil(R / C) + conv)


@dataclass(frozen=True)
class Piece:
    """One work unit: utterance `utt`, chunks [p0, p1) of its chunk grid computed, chunks
    [k0, k1) kept.  Input fbank frames [frame0, frame0 + frames) of the utterance; kept output
    rows land at subsampled frames [row0, row0 + rows) of the utterance."""
    utt: int
    p0: int
    p1: int
    k0: int
    k1: int
    frame0: int
    frames: int
    row0: int
    rows: int
    skip: int          # kept rows start `skip` rows into the piece's output

    @property
    def chunks(self) -> int:
        return self.p1 - self.p0


def _piece(u: int, T: int, C: int, p0: int, p1: int, k0: int, k1: int) -> Piece:
    n = chunks_of(T, C)
    f0 = p0 * 8 * C
    f1 = T if p1 >= n else min(T, p1 * 8 * C + 7)   # + the 7 frames of subsampling overlap
    r0 = k0 * C
    r1 = min(k1 * C, out_len(T))
    return Piece(u, p0, p1, k0, k1, f0, f1 - f0, r0, max(0, r1 - r0), (k0 - p0) * C)


def _lpt(items: Sequence[Tuple[int, int]], world: int, loads: List[int]) -> List[List[int]]:
    """Longest-processing-time placement of (cost, id) items onto ranks with starting `loads`
    (updated in place); returns the ids per rank."""
    heap = [(loads[r], r) for r in range(world)]
    heapq.heapify(heap)
    out: List[List[int]] = [[] for _ in range(world)]
    for w, i in sorted(items, key=lambda x: (-x[0], x[1])):
        load, r = heapq.heappop(heap)
        out[r].append(i)
        loads[r] = load + w
        heapq.heappush(heap, (loads[r], r))
    return out


def _water_fill(long: Sequence[Tuple[int, int]], loads: Sequence[int], level: int, hl: int, hr: int,
                min_keep: int):
    """Cut the long utterances [(u, n)] into consecutive pieces that top every rank up to `level`
    chunks (halos included), least-loaded rank first.  Returns ([(rank, u, k0, k1)], all placed)."""
    order = sorted(range(len(loads)), key=lambda r: (loads[r], r))
    q = [[u, n, 0] for u, n in long]
    placed = []
    for r in order:
        cap = level - loads[r]
        while q and cap > 0:
            u, n, c = q[0]
            lh = min(c, hl)
            if lh + (n - c) <= cap:
                k = n - c
            else:
                k = cap - lh - hr
                if k < min_keep:
                    break
            placed.append((r, u, c, c + k))
            cap -= lh + k + min(n - c - k, hr)
            q[0][2] = c + k
            if c + k == n:
                q.pop(0)
    return placed, not q


def plan_shards(lens: Sequence[int], world: int, C: int = 64, L: int = 128, R: int = 128, num_blocks: int = 12,
                halo: Optional[int] = None, split: bool = True, min_keep: int = 8) -> List[List[Piece]]:
    """Pieces per rank.  Utterances of at most the even share ceil(sum / world) chunks are placed
    whole by LPT; longer ones are then cut on their chunk grid into consecutive pieces that fill
    every rank up to one common level (the lowest level at which everything fits, found by
    bisection), each piece computed with `halo` extra chunks per side (default: the exact receptive
    field, receptive_halo) and at least `min_keep` kept chunks.  Each rank's list is ordered by
    (utterance, first kept chunk)."""
    lens = [int(t) for t in lens]
    world = max(1, int(world))
    n = [chunks_of(t, C) for t in lens]
    if halo is None:
        hl, hr = receptive_halo(C, L, R, num_blocks)
    else:
        hl = hr = int(halo)
    share = max(1, math.ceil(sum(n) / world))
    cut = split and world > 1
    whole = [(nu, u) for u, nu in enumerate(n) if not cut or nu <= share]
    long = [(u, nu) for u, nu in enumerate(n) if cut and nu > share]
    loads = [0] * world
    out: List[List[Piece]] = [[_piece(u, lens[u], C, 0, n[u], 0, n[u]) for u in ids]
                              for ids in _lpt(whole, world, loads)]
    if long:
        need = sum(nu for _, nu in long)
        lo = max(max(loads), math.ceil((sum(loads) + need) / world))
        hi = max(loads) + need + hl + hr + min_keep
        while lo < hi:   # lowest fill level that places every long chunk
            mid = (lo + hi) // 2
            if _water_fill(long, loads, mid, hl, hr, min_keep)[1]:
                hi = mid
            else:
                lo = mid + 1
        placed, ok = _water_fill(long, loads, lo, hl, hr, min_keep)
        assert ok
        for r, u, k0, k1 in placed:
            out[r].append(_piece(u, lens[u], C, max(0, k0 - hl), min(n[u], k1 + hr), k0, k1))
    return [sorted(o, key=lambda p: (p.utt, p.k0)) for o in out]


def lpt_shard(lens: Sequence[int], world: int, C: int = 64) -> List[List[int]]:
    """Whole-utterance LPT assignment (no cuts): per-rank lists of utterance indices."""
    return [[p.utt for p in s] for s in plan_shards(lens, world, C, split=False)]


def rank_rows(shard: Sequence[Piece]) -> int:
    return sum(p.rows for p in shard)


def run_pieces(encoder, xs: Sequence[torch.Tensor], shard: Sequence[Piece], C: int, L: int, R: int,
               want_ids: bool = True, want_logp: bool = False):
    """One masked-batch encoder call over the rank's pieces (features xs[u] [T_u, 80] already on the
    device), then the CTC head.  Returns (kept encoder rows [rows, d], kept ids [rows] int32 or None,
    kept log-probs [rows, V] or None), rows concatenated in shard order."""
    if not shard:
        d = encoder.cfg.d_model
        dev = encoder.device
        return (torch.zeros(0, d, device=dev), torch.zeros(0, dtype=torch.int32, device=dev) if want_ids else None,
                torch.zeros(0, encoder.cfg.vocab, device=dev) if want_logp else None)
    feats = [xs[p.utt][p.frame0: p.frame0 + p.frames] for p in shard]
    lens = torch.tensor([p.frames for p in shard], dtype=torch.int32)
    out, _, n_chunks, _, _, _ = encoder.forward_parallel_chunk(feats, lens, C, L, R)
    flat = out.reshape(-1, out.shape[-1])
    starts = np.cumsum([0] + [nc * C for nc in n_chunks])
    idx = np.concatenate([np.arange(s + p.skip, s + p.skip + p.rows) for s, p in zip(starts, shard)])
    kept = flat.index_select(0, torch.from_numpy(idx).to(flat.device))
    logp, ids = encoder.ctc_log_softmax(kept, want_logp=want_logp, want_ids=want_ids) if (want_ids or want_logp) \
        else (None, None)
    return kept, ids, logp


def assemble_index(shards: List[List[Piece]], lens: Sequence[int], mx: int) -> Tuple[np.ndarray, List[int]]:
    """Source row, in the gathered [world * mx] buffer, of every output row of the batch (the
    utterances' rows concatenated in utterance order), and the per-utterance row counts.  Every row
    of every utterance is kept by exactly one piece of a plan_shards plan."""
    out_lens = [out_len(t) for t in lens]
    starts = np.cumsum([0] + out_lens)
    idx = np.full(int(starts[-1]), -1, np.int64)
    for r, shard in enumerate(shards):
        o = r * mx
        for p in shard:
            d0 = int(starts[p.utt]) + p.row0
            idx[d0: d0 + p.rows] = np.arange(o, o + p.rows)
            o += p.rows
    if (idx < 0).any():
        raise ValueError("the shard plan does not keep every output row")
    return idx, out_lens


_INDEX_CACHE: Dict[tuple, Tuple[torch.Tensor, List[int]]] = {}


def _assemble(buf: torch.Tensor, shards: List[List[Piece]], n_utt: int, lens: Sequence[int]) -> List[torch.Tensor]:
    """buf [world, max_rows, ...] -> per-utterance tensors [out_len(T_u), ...]: ONE index_select
    over the gathered rows with an index built once per plan (kept on buf's device), then views."""
    key = (tuple(tuple(s) for s in shards), tuple(int(t) for t in lens[:n_utt]), buf.shape[1], str(buf.device))
    hit = _INDEX_CACHE.get(key)
    if hit is None:
        idx, out_lens = assemble_index(shards, lens[:n_utt], buf.shape[1])
        if len(_INDEX_CACHE) >= 8:
            _INDEX_CACHE.clear()
        hit = _INDEX_CACHE[key] = (torch.from_numpy(idx).to(buf.device), out_lens)
    idx, out_lens = hit
    flat = buf.reshape((-1,) + tuple(buf.shape[2:])).index_select(0, idx)
    return list(flat.split(out_lens))


def _comm_device(t: torch.Tensor, group) -> torch.device:
    """RCCL ("nccl") works on device tensors; the gloo backend (CPU tests, single-GPU rehearsal
    of several ranks) on host tensors."""
    return t.device if dist.get_backend(group) == "nccl" else torch.device("cpu")


def gather_ids(ids_local: torch.Tensor, shards: List[List[Piece]], lens: Sequence[int], group=None
               ) -> List[torch.Tensor]:
    """The one collective: all_gather_into_tensor of every rank's kept CTC ids (int32, in shard
    order, padded to the largest rank's row count -- known locally from the plan).  Returns the
    per-utterance id tensors of the WHOLE batch, in utterance order, on every rank."""
    world = dist.get_world_size(group)
    dev = _comm_device(ids_local, group)
    mx = max(1, max(rank_rows(s) for s in shards))
    buf = torch.zeros(mx, dtype=torch.int32, device=dev)
    buf[: ids_local.numel()] = ids_local.reshape(-1).to(dev, torch.int32)
    out = torch.empty(world * mx, dtype=torch.int32, device=dev)
    dist.all_gather_into_tensor(out, buf, group=group)
    return _assemble(out.view(world, mx), shards, len(lens), lens)


def gather_logp(logp_local: torch.Tensor, shards: List[List[Piece]], lens: Sequence[int], group=None
                ) -> List[torch.Tensor]:
    """bf16 CTC log-probs of the whole batch on every rank (one all_gather_into_tensor of
    [max_rows, V] bf16 per rank); per-utterance [out_len, V] tensors."""
    world = dist.get_world_size(group)
    dev = _comm_device(logp_local, group)
    V = logp_local.shape[-1]
    mx = max(1, max(rank_rows(s) for s in shards))
    buf = torch.zeros(mx, V, dtype=torch.bfloat16, device=dev)
    buf[: logp_local.shape[0]] = logp_local.to(dev, torch.bfloat16)
    out = torch.empty(world * mx, V, dtype=torch.bfloat16, device=dev)
    dist.all_gather_into_tensor(out, buf, group=group)
    return _assemble(out.view(world, mx, V), shards, len(lens), lens)


def init_from_env(backend: str = None) -> Tuple[int, int, int]:
    """Initialise torch.distributed from torchrun's env (RANK/WORLD_SIZE/LOCAL_RANK/MASTER_*);
    returns (rank, world, local_rank).  Single process without env -> (0, 1, 0), no group.
    Backend: RCCL ("nccl") with a GPU, else gloo; CFM_DIST_BACKEND=gloo forces gloo (several ranks
    rehearsed on one GPU: the collectives then run on host copies)."""
    import os
    if "WORLD_SIZE" not in os.environ or int(os.environ["WORLD_SIZE"]) == 1:
        return 0, 1, int(os.environ.get("LOCAL_RANK", 0))
    rank, world, local = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"]), int(os.environ.get("LOCAL_RANK", 0))
    if backend is None:
        backend = os.environ.get("CFM_DIST_BACKEND") or ("nccl" if torch.cuda.is_available() else "gloo")
    if backend == "nccl":
        torch.cuda.set_device(local)
    dist.init_process_group(backend=backend)
    return rank, world, local
