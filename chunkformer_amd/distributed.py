"""Multi-GPU masked-batch scheduling: one process per GPU, torch.distributed over RCCL.

The reference has no inference-time distribution; this is the
build's own component.  Utterances of a masked batch are independent
(batch-composition invariance), so the packed chunk stream is cut
at utterance boundaries with NO exchange during the encoder:

  lpt_shard      LPT bin-packing of per-utterance chunk counts over the ranks
  gather_ids     the one collective: all_gather of per-rank CTC ids (int32,
                 padded to the max row count) over RCCL/xGMI, reassembled in the
                 original utterance order on every rank
"""
from __future__ import annotations

import heapq
from typing import List, Sequence, Tuple

import torch
import torch.distributed as dist


def chunks_of(T: int, C: int) -> int:
    """n_chunk of one utterance (encoder.py:556-562)."""
    size, step = (C - 1) * 8 + 15, 8 * C
    n_pad = (step - ((T - size) % step)) % step if T >= size else size - T
    return (T + n_pad - size) // step + 1


def lpt_shard(lens: Sequence[int], world: int, C: int = 64) -> List[List[int]]:
    """Longest-processing-time assignment of utterances to `world` ranks by chunk count.
    Returns per-rank lists of utterance indices (each sorted ascending)."""
    work = sorted(((chunks_of(int(t), C), i) for i, t in enumerate(lens)), key=lambda x: (-x[0], x[1]))
    heap = [(0, r) for r in range(world)]
    out: List[List[int]] = [[] for _ in range(world)]
    for w, i in work:
        load, r = heapq.heappop(heap)
        out[r].append(i)
        heapq.heappush(heap, (load + w, r))
    return [sorted(o) for o in out]


def gather_ids(ids_local: torch.Tensor, lens_local: Sequence[int], shards: List[List[int]], group=None
               ) -> List[torch.Tensor]:
    """All-gather per-utterance CTC ids.

    ids_local: [rows_local] int32, the local utterances' frames concatenated in shard order
    (utterance k contributes lens_local[k] rows).  Returns the list of per-utterance id
    tensors for the WHOLE batch, in original utterance order, on every rank."""
    world = dist.get_world_size(group)
    rows = torch.tensor([ids_local.numel()], dtype=torch.int64, device=ids_local.device)
    all_rows = [torch.zeros_like(rows) for _ in range(world)]
    dist.all_gather(all_rows, rows, group=group)
    mx = int(max(int(r.item()) for r in all_rows))
    buf = torch.zeros(max(mx, 1), dtype=torch.int32, device=ids_local.device)
    buf[: ids_local.numel()] = ids_local.to(torch.int32)
    out = torch.empty(world * buf.numel(), dtype=torch.int32, device=ids_local.device)
    dist.all_gather_into_tensor(out, buf, group=group)
    out = out.view(world, -1)
    n_utt = sum(len(s) for s in shards)
    res: List[torch.Tensor] = [None] * n_utt  # type: ignore
    # per-rank utterance lengths are needed to cut; exchange them too (tiny)
    lens_t = torch.zeros(n_utt, dtype=torch.int64, device=ids_local.device)
    me = dist.get_rank(group)
    for k, u in enumerate(shards[me]):
        lens_t[u] = int(lens_local[k])
    dist.all_reduce(lens_t, group=group)
    lens_all = lens_t.tolist()
    for r, shard in enumerate(shards):
        o = 0
        for u in shard:
            res[u] = out[r, o: o + lens_all[u]]
            o += lens_all[u]
    return res


def init_from_env(backend: str = None) -> Tuple[int, int, int]:
    """Initialise torch.distributed from torchrun's env (RANK/WORLD_SIZE/LOCAL_RANK/MASTER_*);
    returns (rank, world, local_rank).  Single process without env -> (0, 1, 0), no group."""
    import os
    if "WORLD_SIZE" not in os.environ or int(os.environ["WORLD_SIZE"]) == 1:
        return 0, 1, int(os.environ.get("LOCAL_RANK", 0))
    rank, world, local = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"]), int(os.environ.get("LOCAL_RANK", 0))
    if backend is None:
        backend = "nccl" if torch.cuda.is_available() else "gloo"
    if backend == "nccl":
        torch.cuda.set_device(local)
    dist.init_process_group(backend=backend)
    return rank, world, local
