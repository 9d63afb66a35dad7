"""Multi-rank scheduling on CPU (gloo, world_size 2): utterance sharding of the masked
batch (LPT over chunk counts) and the one collective, the CTC-id all-gather
(chunkformer_amd/distributed.py).  The GPU run uses the same code over RCCL."""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from chunkformer_amd.distributed import chunks_of, gather_ids, lpt_shard


def test_chunks_of_matches_planner():
    from oracle.encoder_ref import plan_utterance
    for T in (1, 14, 15, 518, 519, 520, 1031, 1032, 100_000):
        assert chunks_of(T, 64) == plan_utterance(T, 64)[1]


def test_lpt_shard_partition_and_balance():
    import random
    rnd = random.Random(0)
    lens = [rnd.randint(100, 180_000) for _ in range(284)]
    for world in (1, 2, 3, 8):
        sh = lpt_shard(lens, world)
        flat = sorted(i for s in sh for i in s)
        assert flat == list(range(len(lens)))
        loads = [sum(chunks_of(lens[i], 64) for i in s) for s in sh]
        assert max(loads) - min(loads) <= max(chunks_of(t, 64) for t in lens)
    assert lpt_shard([10, 10], 4)[2:] == [[], []]


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, lens, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        shards = lpt_shard(lens, world)
        mine = shards[rank]
        # fake "CTC ids": utterance u contributes lens[u] rows filled with u*1000 + frame
        ids = torch.cat([torch.arange(lens[u], dtype=torch.int32) + 1000 * u for u in mine]) if mine else \
            torch.zeros(0, dtype=torch.int32)
        res = gather_ids(ids, [lens[u] for u in mine], shards)
        ok = all(torch.equal(res[u], torch.arange(lens[u], dtype=torch.int32) + 1000 * u) for u in range(len(lens)))
        q.put((rank, ok))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("lens", [[5, 17, 3, 40, 8, 1], [7]])
def test_gather_ids_world2(lens):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_worker, args=(r, 2, port, lens, q)) for r in range(2)]
    for p in ps:
        p.start()
    for p in ps:
        p.join(120)
    res = dict(q.get(timeout=5) for _ in range(2))
    assert res == {0: True, 1: True}
    assert all(p.exitcode == 0 for p in ps)
