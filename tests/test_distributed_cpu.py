"""Multi-rank scheduling on CPU (gloo, world_size 2): the shard plan of the masked batch
(LPT pieces, utterances longer than a rank's share cut with halos) and the one collective,
the CTC-id all-gather with per-utterance reassembly across cuts
(chunkformer_amd/distributed.py).  The GPU run uses the same code over RCCL."""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from chunkformer_amd.distributed import (chunks_of, gather_ids, gather_logp, lpt_shard, out_len, plan_shards,
                                         receptive_halo)


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


@pytest.mark.parametrize("world", [1, 2, 3, 8])
@pytest.mark.parametrize("case", ["bench980", "skewed", "tiny"])
def test_plan_shards_partition(world, case):
    """Kept chunks of every utterance tile [0, n) exactly once, kept rows tile [0, calc_length(T)),
    every piece's input window sits on the utterance's chunk grid (8C frames per chunk, + 7 frames
    of subsampling overlap) with the halo clipped to the utterance, and the loads are balanced."""
    import math
    import random
    C = 64
    if case == "bench980":
        rnd = random.Random(0)
        lens, tot = [], 0
        while tot < 980 * 6000:
            T = min(int(math.exp(math.log(100) + rnd.random() * (math.log(180000) - math.log(100)))), 980 * 6000 - tot)
            lens.append(T)
            tot += T
    elif case == "skewed":
        lens = [5_760_000, 123_457] + [3000 + 17 * i for i in range(60)]
    else:
        lens = [1, 14, 15, 519, 520, 1031, 1032, 1039]
    sh = plan_shards(lens, world)
    hl, hr = receptive_halo(C, 128, 128, 12)
    kept = {u: [] for u in range(len(lens))}
    for shard in sh:
        for p in shard:
            n = chunks_of(lens[p.utt], C)
            assert 0 <= p.p0 <= p.k0 < p.k1 <= p.p1 <= n
            assert p.k0 - p.p0 == min(p.k0, hl) and p.p1 - p.k1 == min(n - p.k1, hr)
            assert p.frame0 == p.p0 * 8 * C
            assert chunks_of(p.frames, C) == p.p1 - p.p0
            assert p.skip == (p.k0 - p.p0) * C
            kept[p.utt].append(p)
    for u, ps in kept.items():
        ps.sort(key=lambda p: p.k0)
        n = chunks_of(lens[u], C)
        assert ps[0].k0 == 0 and ps[-1].k1 == n
        assert all(a.k1 == b.k0 for a, b in zip(ps, ps[1:]))
        assert sum(p.rows for p in ps) == out_len(lens[u])
        assert all(a.row0 + a.rows == b.row0 for a, b in zip(ps, ps[1:]))
    loads = [sum(p.chunks for p in s) for s in sh]
    total = sum(chunks_of(t, C) for t in lens)
    if case == "bench980":
        assert max(loads) <= total / world + 344   # no cuts needed, LPT within one utterance
    if case == "skewed" and world > 1:
        assert max(loads) <= 1.05 * sum(loads) / world   # the 16 h file is cut: balanced
    if world == 1:
        assert all(p.k0 == 0 and p.k1 == chunks_of(lens[p.utt], C) for p in sh[0])


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _fake_ids(u, rows):
    """fake "CTC ids" of utterance u's subsampled frames `rows` (what the encoder + CTC head would
    give for them; a halo cut must not change them)"""
    return rows.to(torch.int32) * 7 + 100_000 * u


def _worker(rank, world, port, lens, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        shards = plan_shards(lens, world, C=16, L=32, R=32, num_blocks=2)
        mine = shards[rank]
        parts = [_fake_ids(p.utt, torch.arange(p.row0, p.row0 + p.rows)) for p in mine]
        ids = torch.cat(parts) if parts else torch.zeros(0, dtype=torch.int32)
        res = gather_ids(ids, shards, lens)
        ok = all(torch.equal(res[u], _fake_ids(u, torch.arange(out_len(lens[u])))) for u in range(len(lens)))
        # the bf16 log-prob gather: rows of V=3 values derived from the same ids
        lp = torch.stack([ids.float(), -ids.float(), ids.float() / 3], 1) if ids.numel() else torch.zeros(0, 3)
        lres = gather_logp(lp, shards, lens)
        for u in range(len(lens)):
            e = _fake_ids(u, torch.arange(out_len(lens[u]))).float()
            ok = ok and torch.equal(lres[u], torch.stack([e, -e, e / 3], 1).to(torch.bfloat16))
        cut = any(p.k0 > 0 for s in shards for p in s)
        q.put((rank, (ok, cut)))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("lens,cut", [([5000, 170, 30, 4000, 800, 15], False), ([70], False),
                                      ([60_000, 500, 300, 200], True), ([9000, 9000, 20], False)])
def test_gather_ids_world2(lens, cut):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_worker, args=(r, 2, port, lens, q)) for r in range(2)]
    for p in ps:
        p.start()
    for p in ps:
        p.join(120)
    res = dict(q.get(timeout=5) for _ in range(2))
    assert res == {0: (True, cut), 1: (True, cut)}
    assert all(p.exitcode == 0 for p in ps)
