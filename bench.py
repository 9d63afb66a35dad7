"""Benchmark: audio-frames/s through the ChunkFormer encoder (masked batch) on MI355X.

    python bench.py --gpus N --steps K --warmup W

N > 1: either launched by `python -m torch.distributed.run --nproc-per-node N bench.py --gpus N`
(WORLD_SIZE must equal N, else the run exits non-zero), or started plainly, in which case bench.py
starts that torch.distributed.run itself as a child process before any GPU call, relays its
output and exits with its return code.

Workload: chunkformer-large (12 layers, d=512, 8 heads, ff=2048, conv k=15,
V=5000) with seeded synthetic weights, synthetic N(0,1) 80-dim fbank, utterance lengths
log-uniform in [1 s, 30 min] from torch.Generator seed 0, chunk 64 / left 128 / right 128.

  --config auto (default): masked at N = 1, sharded at N > 1
  --config masked   BASELINE configs[1]: a 240-min masked batch (B=70, N=2,845 chunks) PER GPU
                    (weak scaling)
  --config sharded  BASELINE configs[2]: ONE 980-min masked batch (B=284, N=11,625 chunks)
                    sharded over the ranks (strong scaling): distributed.plan_shards cuts it into
                    per-rank pieces (LPT over chunk counts; utterances longer than a rank's share
                    are split with recomputed halos), no exchange during the encoder; after timing
                    the CTC ids (fused argmax head) go through ONE all_gather_into_tensor over
                    RCCL/xGMI, and the bf16 log-probs through another, each timed separately
  --config endless / full   configs[3] / configs[4] (one GPU)

A step = ChunkFormerEncoder.forward_parallel_chunk over the rank's whole batch:
host packer (C++ planner) + plan upload + front-end + 12 blocks + after_norm, with
the features already resident in HBM.  value = all ranks' fbank frames / max-over-
ranks step time.

roofline: the dominant kernel is the FFN w_1 GEMM with its fused bias + SiLU epilogue
(2 x 64N x 512 x 2048 FLOP per launch); its per-launch time is measured live with HIP events on
the launch stream (libcfm in-stream profiler) over the timed steps.  end_to_end_ms: the same step
plus the fused CTC ids head and, at N > 1, the ids all-gather (max over ranks).  cpu_baseline:
the CPU oracle (oracle/encoder_ref.py, torch fp32) on a bounded sample of the same workload, and
on one 30 s utterance (configs[0]).
"""
from __future__ import annotations

import argparse
import json
import math
import os
import sys
import time

import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

from chunkformer_amd import _lib  # noqa: E402
from chunkformer_amd.config import LARGE  # noqa: E402
from chunkformer_amd.distributed import (_assemble, chunks_of, gather_ids, gather_logp, init_from_env,  # noqa: E402
                                         plan_shards, rank_rows)
from chunkformer_amd.encoder import ChunkFormerEncoder  # noqa: E402
from chunkformer_amd.weights import synthetic_state_dict  # noqa: E402

METRIC = "audio-frames/sec (80-dim fbank) through encoder, chunkformer-large chunk=64, 1/2/4/8 GPU"
PEAK_TFLOPS = {"bf16": 2500.0, "fp16": 2500.0, "fp32": 157.3}   # MI355X dense MFMA peaks (MI355X_MICROARCH.md)
MEASURED_BF16_CEILING = 1833.8   # TFLOP/s, tools/mfma_peak.hip on this pool
HIPBLASLT_W1 = 706.8             # TFLOP/s, hipBLASLt M=182080 N=2048 K=512 bf16
C, L, R = 64, 128, 128
# fbank, 25 ms / 10 ms at 16 kHz (win 400, N = 512, M = 256 complex points, 80 bins): 5 FLOP per
# sample of frame preparation (mean, DC, pre-emphasis, window), 5 M log2 M for the complex FFT,
# 13 per bin for the real split and |X|^2, 2 per filter weight (each of the 257 bins in <= 2 filters)
FBANK_FLOPS_PER_FRAME = 5 * 400 + 5 * 256 * 8 + 13 * 257 + 2 * 2 * 257


def workload_lengths(total_frames: int, seed: int = 0):
    """SURVEY §8d generator: log-uniform 1 s .. 30 min until the target is reached."""
    g = torch.Generator().manual_seed(seed)
    lens, tot = [], 0
    lo, hi = math.log(100), math.log(180000)
    while tot < total_frames:
        T = int(math.exp(lo + float(torch.rand(1, generator=g)) * (hi - lo)))
        T = min(T, total_frames - tot)
        lens.append(T)
        tot += T
    return lens


def flops_per_chunk(cfg) -> float:
    """Algorithmic FLOPs of one 64-frame chunk."""
    d, ff, k = cfg.d_model, cfg.ffn_dim, cfg.kernel_size
    front = 2 * (d * (4 * C + 3) * 39 * 9 + d * (2 * C + 1) * 19 * 9 + d * d * (2 * C + 1) * 19 + d * C * 9 * 9
                 + d * d * C * 9 + C * 9 * d * d)
    layer = 2 * (2 * 2 * C * d * ff + 4 * C * d * d + 2 * C * d * d + C * d * d + C * d * k
                 + C * d * (L + C + R) + C * d * (L + 2 * C + R - 1) + C * d * (L + C + R))
    return front + cfg.num_blocks * layer


def host_cpu():
    """(CPU model, physical cores this process may run on): /proc/cpuinfo over the affinity set,
    capped by the box's thread share (OMP_NUM_THREADS) when it is set."""
    allowed = set(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else set(range(os.cpu_count() or 1))
    model, cores, cur = "unknown", set(), {}
    try:
        with open("/proc/cpuinfo") as f:
            lines = f.read().split("\n") + [""]
    except OSError:
        lines = []
    for line in lines:
        if not line.strip():
            if cur.get("processor", "").isdigit() and int(cur["processor"]) in allowed:
                cores.add((cur.get("physical id", "0"), cur.get("core id", cur["processor"])))
                model = cur.get("model name", model)
            cur = {}
            continue
        k, _, v = line.partition(":")
        cur[k.strip()] = v.strip()
    n = len(cores) or len(allowed)
    cap = os.environ.get("OMP_NUM_THREADS", "")
    if cap.isdigit() and int(cap) > 0:
        n = min(n, int(cap))
    return model, max(1, n)


def cpu_baseline(lens_all, budget_s: float = 12.0):
    """Time the CPU oracle (torch fp32) on consecutive utterance groups until the budget, on every
    physical core of the process's CPU share."""
    from chunkformer_amd.weights import synthetic_features
    from oracle import encoder_ref as ref
    model, threads = host_cpu()
    torch.set_num_threads(threads)
    sd = synthetic_state_dict(LARGE, 0)
    frames, t_tot, groups, i = 0, 0.0, 0, 0
    while t_tot < budget_s and i < len(lens_all):
        grp = []
        while i < len(lens_all) and sum(grp) < 30000:
            grp.append(min(lens_all[i], 60000))
            i += 1
        xs = synthetic_features(grp, 1000 + groups)
        t0 = time.perf_counter()
        ref.forward_parallel_chunk(sd, LARGE, xs, grp, C, L, R)
        t_tot += time.perf_counter() - t0
        frames += sum(grp)
        groups += 1
    # configs[0]: one 30 s utterance (3000 frames, 6 chunks) through the same oracle call
    x1 = synthetic_features([3000], 999)
    ref.forward_parallel_chunk(sd, LARGE, x1, [3000], C, L, R)   # untimed first call
    t1, reps = 0.0, 0
    while t1 < 3.0 and reps < 20:
        c0 = time.perf_counter()
        ref.forward_parallel_chunk(sd, LARGE, x1, [3000], C, L, R)
        t1 += time.perf_counter() - c0
        reps += 1
    return {"value": round(frames / t_tot, 1), "unit": "audio-frames/s", "cores": threads, "cpu": model,
            "kind": "port",
            "sample": f"{groups} masked-batch calls of the oracle (oracle/encoder_ref.py, torch fp32 CPU) over the "
                      f"workload's first utterances (capped at 60k frames each), {frames} frames in {t_tot:.1f} s",
            "config1_30s_utterance": {"value": round(3000 * reps / t1, 1), "unit": "audio-frames/s",
                                      "ms_per_utterance": round(t1 / reps * 1e3, 1), "reps": reps}}


def newest_profile(kind: str):
    """The committed profile summary profiles/r<NN>[_final]_<kind>.json of the latest round (the round's
    final-build profile over its earlier ones): ordered by round number, not by name ('f' < 't' made a
    name sort pick an earlier build's file); None if absent."""
    import glob
    import re
    best, key = None, None
    for f in glob.glob(os.path.join(ROOT, "profiles", f"r*_{kind}.json")):
        m = re.match(r"r(\d+)(_final)?_" + kind + r"\.json$", os.path.basename(f))
        if m and (key is None or (int(m.group(1)), bool(m.group(2))) > key):
            best, key = f, (int(m.group(1)), bool(m.group(2)))
    return best


def committed_traffic(cls: str = "ffn_w1_gemm"):
    """HBM bytes per launch of the roofline kernel from the newest committed PMC summary
    (profiles/<round>_traffic.json, made by tools/profile_round.sh with rocprofv3
    FETCH_SIZE/WRITE_SIZE passes on this same workload); None if absent."""
    f = newest_profile("traffic")
    if not f:
        return None, None
    try:
        ent = json.load(open(f))["kernels"].get(cls)
        return (float(ent[0]["hbm_bytes_per_launch"]), os.path.relpath(f, ROOT)) if ent else (None, None)
    except (OSError, ValueError, KeyError, IndexError):
        return None, None


def committed_mfma_busy(cls: str = "ffn_w1_gemm"):
    """MFMA busy fraction and effective clock of the roofline kernel from the newest committed PMC
    summary (profiles/<round>_mfma_busy.json, tools/profile_round.sh: GRBM_GUI_ACTIVE +
    SQ_VALU_MFMA_BUSY_CYCLES over this same workload); (None, None, None) if absent."""
    f = newest_profile("mfma_busy")
    if not f:
        return None, None, None
    try:
        ent = json.load(open(f))["kernels"].get(cls)
        return ((ent["mfma_busy"], ent["clock_ghz"], os.path.relpath(f, ROOT)) if ent else (None, None, None))
    except (OSError, ValueError, KeyError):
        return None, None, None


def class_rooflines(prof, n_chunks: int, cfg, dtype: str, profiled: bool):
    """Per kernel class of one profiled step: ms, launches and the roofline fraction -- MFMA classes
    against the dense peak from their algorithmic FLOPs (SURVEY 8(d) per-chunk terms), HBM classes
    against 8 TB/s from the committed PMC bytes per launch (only on the profiled workload)."""
    d, ff, nb, Cc = cfg.d_model, cfg.ffn_dim, cfg.num_blocks, C
    rows = n_chunks * Cc
    W = L + Cc + R
    flops = {
        "ffn_w1_gemm": 2.0 * rows * ff * d * 2 * nb, "ffn_w2_gemm": 2.0 * rows * ff * d * 2 * nb,
        "qkv_gemm": 2.0 * rows * 3 * d * d * nb, "out_proj_gemm": 2.0 * rows * d * d * nb,
        "pw1_glu_gemm": 2.0 * rows * 2 * d * d * nb, "pw2_gemm": 2.0 * rows * d * d * nb,
        "chunk_attention": 2.0 * n_chunks * Cc * d * (W + (L + 2 * Cc + R - 1) + W) * nb,
        "frontend_pw_gemm": 2.0 * n_chunks * (d * d * (2 * Cc + 1) * 19 + d * d * Cc * 9 + Cc * 9 * d * d),
    }
    hbm = {"layernorm": ("layernorm", "layernorm2"), "frontend_dw2": ("frontend_dw2",),
           "conv_dw_ln_silu": ("conv_dw_ln_silu",), "frontend_conv0_dw": ("frontend_conv0_dw",)}
    traffic = {}
    if profiled:
        f = newest_profile("traffic")
        if f:
            try:
                traffic = json.load(open(f))["kernels"]
            except (OSError, ValueError, KeyError):
                traffic = {}
    out = {}
    for cls, (ms, n) in prof.items():
        if not n:
            continue
        ent = {"ms_per_step": round(ms, 3), "launches": n}
        if cls in flops:
            ach = flops[cls] / (ms / 1e3) / 1e12
            ent.update(bound="mfma", achieved_tflops=round(ach, 1), frac=round(ach / PEAK_TFLOPS[dtype], 3))
        elif cls in hbm and traffic:
            # PMC bytes per launch x launches of each kernel of the class (LN: ln_kernel and ln2_kernel)
            tot = sum(e["hbm_bytes_per_launch"] * e["dispatches"] for k in hbm[cls] for e in traffic.get(k, []))
            disp = sum(e["dispatches"] for k in hbm[cls] for e in traffic.get(k, []))
            if disp:
                per_step = tot / disp * n
                ach = per_step / (ms / 1e3) / 1e9
                ent.update(bound="hbm", achieved_gbs=round(ach, 1), frac=round(ach / 8000.0, 3),
                           pmc_bytes_per_step=round(per_step))
        out[cls] = ent
    return out


def apply_opts(enc, opts):
    for kv in opts:
        k, v = kv.split("=")
        enc.set_option(k, int(v, 0))


def spawn_ranks(n: int) -> int:
    """--gpus N > 1 without a torchrun environment: run `python -m torch.distributed.run
    --nproc-per-node N bench.py <same args>` as a child process (this process has not touched the
    GPU), its rank 0 printing the JSON line on the inherited stdout; returns its exit code."""
    import socket
    import subprocess
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr", "127.0.0.1", f"--master-port={port}", os.path.abspath(__file__), *sys.argv[1:]]
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    return subprocess.call(cmd, env=env)


def model_config(heads: int):
    """chunkformer-large (8 heads, BASELINE configs) or its 4-head d=512 variant (head_dim 128,
    the reference's shipped recipes, examples/asr/rnnt/conf/chunkformer-rnnt-large-vie.yaml:5-6)."""
    from chunkformer_amd.config import LARGE_4H
    if heads == 8:
        return LARGE
    if heads == 4:
        return LARGE_4H
    raise SystemExit("--heads must be 8 or 4")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--dtype", default="bf16", choices=["bf16", "fp16", "fp32"])
    ap.add_argument("--minutes", type=float, default=None,
                    help="audio minutes: per GPU for masked (240), of the whole batch for sharded (980)")
    ap.add_argument("--no-gather-logp", action="store_true", help="sharded: skip the bf16 log-prob all-gather")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-breakdown", action="store_true")
    ap.add_argument("--config", default="auto", choices=["auto", "masked", "sharded", "endless", "full", "fbank"],
                    help="auto = masked at 1 GPU, sharded at N > 1; masked = configs[1] (240 min per GPU, the "
                         "headline line); sharded = configs[2] (one 980-min batch over all ranks); endless = "
                         "configs[3] (16 h endless_decode, graph-replayed segments); full = configs[4] (full "
                         "attention, B=256)")
    ap.add_argument("--hours", type=float, default=16.0, help="endless: audio hours")
    ap.add_argument("--endless-mode", default="graphpipe", choices=["graphpipe", "pipeline", "graph"],
                    help="endless: --pipeline-depth segments in flight, every segment (up to 128 per graph) replaying "
                         "one captured HIP graph of that multi-stream pipeline (graphpipe), the same pipeline "
                         "launched eagerly (pipeline), or one segment "
                         "at a time replaying one captured graph per middle segment (graph); all bit-identical "
                         "to the eager loop")
    ap.add_argument("--pipeline-depth", type=int, default=None,
                    help="endless pipeline: segments in flight (default 4 for graphpipe, 3 for pipeline: the "
                         "measured best of each at tbd 1800)")
    ap.add_argument("--tbd", type=int, default=7200,
                    help="endless: total_batch_duration (s); a memory budget that does not change results "
                         "(tests/test_gpu_model.py): 7200 s segments fill one MI355X better than the "
                         "reference's 1800 s default (DESIGN.md §8)")
    ap.add_argument("--batch", type=int, default=256, help="full: utterances of T=3000 frames")
    ap.add_argument("--pipe-opt", action="append", default=[], metavar="KEY=VALUE",
                    help="endless (A/B): override a launch parameter of the segments in flight (streaming.PIPELINE_OPTS)")
    ap.add_argument("--no-fe-reuse", action="store_true",
                    help="endless (A/B): recompute every segment's first front-end windows instead of carrying them")
    ap.add_argument("--opt", action="append", default=[], metavar="KEY=VALUE",
                    help="per-model kernel option (cfm_model_set_option), A/B runs only")
    ap.add_argument("--heads", type=int, default=8, choices=[8, 4],
                    help="attention heads of the d=512 model: 8 (chunkformer-large, BASELINE) or 4 (head_dim 128, "
                         "the reference's shipped d=512 recipes)")
    args = ap.parse_args()
    env_world = int(os.environ.get("WORLD_SIZE", "0") or 0)
    if env_world == 0 and args.gpus > 1:
        if args.config in ("endless", "full", "fbank"):
            raise SystemExit(f"--config {args.config} runs on one GPU")
        sys.exit(spawn_ranks(args.gpus))
    if env_world and env_world != args.gpus:
        raise SystemExit(f"WORLD_SIZE={env_world} but --gpus {args.gpus}: launch one rank per GPU")
    if args.config in ("endless", "full"):
        return bench_single(args)
    if args.config == "fbank":
        return bench_fbank(args)

    rank, world, local = init_from_env()
    ndev = torch.cuda.device_count()
    if world > ndev and (os.environ.get("CFM_DIST_BACKEND") or "nccl") == "nccl":
        raise SystemExit(f"{world} ranks but {ndev} GPU(s): RCCL needs one GPU per rank "
                         "(CFM_DIST_BACKEND=gloo rehearses several ranks on one GPU)")
    local = local % ndev   # (rehearsal of several ranks on one GPU: gloo backend)
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    sharded = args.config == "sharded" or (args.config == "auto" and world > 1)
    minutes = args.minutes if args.minutes is not None else (980.0 if sharded else 240.0)
    cfg = model_config(args.heads)
    if sharded:   # configs[2]: one batch of `minutes` over all ranks
        lens_all = workload_lengths(int(minutes * 60 * 100), seed=0)
        shards = plan_shards(lens_all, world, C, L, R, cfg.num_blocks)
    else:         # configs[1]: `minutes` per rank, whole utterances LPT-placed
        lens_all = workload_lengths(int(minutes * 60 * 100) * world, seed=0)
        shards = plan_shards(lens_all, world, C, L, R, cfg.num_blocks, split=False)
    mine = shards[rank]
    # features: utterance u from its own seed, so every rank sees the same audio for u
    need = sorted({p.utt for p in mine})
    full = {u: torch.randn(lens_all[u], 80, generator=torch.Generator(device=dev).manual_seed(1234 + u), device=dev)
            for u in need}
    xs = [full[p.utt][p.frame0: p.frame0 + p.frames] for p in mine]
    lens = [p.frames for p in mine]
    xs_lens = torch.tensor(lens, dtype=torch.int32)
    n_chunks = sum(chunks_of(t, C) for t in lens)
    # real audio frames this rank answers for: its kept chunks' frames (halo frames recomputed
    # around cuts are not counted); over all ranks this sums to the batch's frames exactly
    real_frames = sum((lens_all[p.utt] if p.k1 == chunks_of(lens_all[p.utt], C) else p.k1 * 8 * C) - p.k0 * 8 * C
                      for p in mine)

    enc = ChunkFormerEncoder(cfg, synthetic_state_dict(cfg, 0), device=dev, dtype=args.dtype)
    apply_opts(enc, args.opt)

    def step():
        return enc.forward_parallel_chunk(xs, xs_lens, C, L, R)

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    roof_bits = 1 << _lib.PROFILE_CLASSES.index("ffn_w1_gemm")
    enc.set_option("profile_reset", 1)
    enc.set_option("profile", roof_bits)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        out = step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    dt = time.perf_counter() - t0
    enc.set_option("profile", 0)
    prof = _lib.profile_read(enc._h)
    t = torch.tensor([dt], dtype=torch.float64, device=dev)
    frames = torch.tensor([float(real_frames)], dtype=torch.float64, device=dev)
    if world > 1:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dist.all_reduce(frames, op=dist.ReduceOp.SUM)
    dt_max = float(t.item())
    total_frames = float(frames.item())
    value = total_frames * args.steps / dt_max

    # ---- dominant kernel: the FFN (fused kernel, or its w_1 GEMM on the two-GEMM path);
    # per-launch time from in-stream HIP events on the launch stream (libcfm profiler)
    rows = n_chunks * C
    d_, ff_ = cfg.d_model, cfg.ffn_dim
    roof_cls = "ffn_w1_gemm"
    roof_name = (f"ffn_w1_gemm (gemm_wsp_kernel<EPI_STORE,SiLU>: K=512 weight-stationary {args.dtype[:2]}16 MFMA)"
                 if args.dtype in ("bf16", "fp16") else "ffn_w1_gemm (gemm_kernel<float,EPI_STORE,SiLU>, exact-f32 MFMA)")
    # per step: one w_1 launch per layer and utterance group (enc.stream_split groups of the batch run
    # on their own streams, so a launch covers rows / groups rows); totals over the timed launches
    # (two FFNs per layer: the macaron and the final one)
    fl_step = 2.0 * rows * ff_ * d_ * 2 * cfg.num_blocks
    ms1, n1 = prof[roof_cls]
    per_step = n1 / args.steps if n1 else 1
    fl_launch = fl_step / per_step
    rows_launch = rows / (per_step / (2 * cfg.num_blocks))
    # compulsory bytes of one w_1 launch: A [rows, d] + out [rows, ff] bf16 + W [ff, d] bf16 + bias
    alg_bytes = 2.0 * (rows_launch * d_ + rows_launch * ff_ + ff_ * d_) + 4 * ff_
    avg_s = (ms1 / max(n1, 1)) / 1e3
    achieved = fl_step * args.steps / (ms1 / 1e3) / 1e12 if n1 else None
    peak = PEAK_TFLOPS[args.dtype]
    # the committed PMC traffic was collected on the default workload (configs[1], 2,845 chunks on one
    # GPU); other row counts report null rather than a number measured on a different launch size
    profiled = (args.dtype == "bf16" and not sharded and world == 1 and n_chunks == 2845 and args.heads == 8
                and per_step == 2 * cfg.num_blocks)   # the committed PMC passes ran un-split launches
    traffic, traffic_src = committed_traffic(roof_cls) if profiled else (None, None)
    busy, busy_clk, busy_src = committed_mfma_busy(roof_cls) if profiled else (None, None, None)
    step_flops = n_chunks * flops_per_chunk(cfg) + cfg.num_blocks * 2 * (L + 2 * C + R - 1) * cfg.d_model ** 2

    # ---- CTC head + the collectives (timed separately; not part of `value`)
    enc_out = out[0]
    enc.ctc_log_softmax(enc_out, want_logp=False)   # first call loads the kernel
    torch.cuda.synchronize()
    tc = time.perf_counter()
    _, ids = enc.ctc_log_softmax(enc_out, want_logp=False)   # fused argmax head (ids only)
    torch.cuda.synchronize()
    ctc_ms = (time.perf_counter() - tc) * 1e3
    gather_ms = gather_lp_ms = None
    # the kept rows of every piece, in shard order (the layout gather_* expects)
    starts = torch.tensor([0] + list(out[2][:-1])).cumsum(0) * C
    idx = torch.cat([torch.arange(int(s) + p.skip, int(s) + p.skip + p.rows) for s, p in zip(starts, mine)]).to(dev)
    if world > 1:
        flat = ids.reshape(-1).index_select(0, idx)
        dist.barrier()
        torch.cuda.synchronize()
        tg = time.perf_counter()
        gather_ids(flat, shards, lens_all)
        torch.cuda.synchronize()
        gather_ms = (time.perf_counter() - tg) * 1e3
        if sharded and not args.no_gather_logp:
            logp, _ = enc.ctc_log_softmax(enc_out.reshape(-1, cfg.d_model).index_select(0, idx), want_logp=True,
                                          want_ids=False)
            dist.barrier()
            torch.cuda.synchronize()
            tg = time.perf_counter()
            gather_logp(logp, shards, lens_all)
            torch.cuda.synchronize()
            gather_lp_ms = (time.perf_counter() - tg) * 1e3
            del logp
    del out, enc_out, ids
    # the gather's per-utterance reassembly at configs[2]'s world 8, timed on this GPU alone: one
    # index_select of the gathered [8, max_rows] ids with the plan's cached index, then views
    assemble_ms = None
    if sharded and rank == 0:
        sh8 = plan_shards(lens_all, 8, C, L, R, cfg.num_blocks)
        buf8 = torch.zeros(8, max(1, max(sum(p.rows for p in s_) for s_ in sh8)), dtype=torch.int32, device=dev)
        _assemble(buf8, sh8, len(lens_all), lens_all)   # builds and uploads the plan's index once
        torch.cuda.synchronize()
        ta = time.perf_counter()
        for _ in range(5):
            _assemble(buf8, sh8, len(lens_all), lens_all)
        torch.cuda.synchronize()
        assemble_ms = (time.perf_counter() - ta) / 5 * 1e3
        del buf8

    # ---- end to end: the step + the fused CTC ids head + (N > 1) the ids all-gather with the
    # per-utterance reassembly on every rank; K steps between barriers, max over ranks
    def e2e():
        o = step()
        _, ids_ = enc.ctc_log_softmax(o[0], want_logp=False)
        if world > 1:
            gather_ids(ids_.reshape(-1).index_select(0, idx), shards, lens_all)
        return ids_
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        e2e()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    te = torch.tensor([time.perf_counter() - t0], dtype=torch.float64, device=dev)
    if world > 1:
        dist.all_reduce(te, op=dist.ReduceOp.MAX)
    e2e_ms = float(te.item()) / args.steps * 1e3

    breakdown = by_class = None
    if not args.no_breakdown:
        enc.set_option("profile_reset", 1)
        enc.set_option("profile", (1 << len(_lib.PROFILE_CLASSES)) - 1)
        step()
        torch.cuda.synchronize()
        enc.set_option("profile", 0)
        prof_all = _lib.profile_read(enc._h)
        breakdown = {k: round(v[0], 3) for k, v in prof_all.items() if v[1]}
        by_class = class_rooflines(prof_all, n_chunks, cfg, args.dtype, profiled)

    if rank == 0:
        res = {
            "metric": METRIC,
            "value": round(value, 1),
            "unit": "audio-frames/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(dt_max / args.steps * 1e3, 3),
            "higher_is_better": True,
            "scaling": "strong" if sharded else "weak",
            "vs_baseline": None,
            "dtype": args.dtype,
            "data": "synthetic (N(0,1) 80-dim fbank, seeded random chunkformer-large weights; no checkpoint offline)",
            "config": {"workload": (f"configs[2]: one {minutes:g}-min masked batch (log-uniform 1 s-30 min utterances, "
                                    f"seed 0, B={len(lens_all)}) sharded over {world} GPU(s) by plan_shards, "
                                    f"forward_parallel_chunk C=64 L=128 R=128" if sharded else
                                    f"configs[1]: masked batch, {minutes:g} min of audio per GPU (log-uniform 1 s-30 "
                                    f"min utterances, seed 0), forward_parallel_chunk C=64 L=128 R=128"),
                       "config_index": 2 if sharded else 1,
                       "heads": cfg.n_heads, "head_dim": cfg.head_dim,
                       "pieces_rank0": len(mine), "chunks_rank0": n_chunks, "frames_total": int(total_frames),
                       "parallelism": f"dp{world} ({'plan_shards: LPT pieces, halo cuts' if sharded else 'LPT utterance sharding'})"},
            # ranks vs physical GPUs: world > devices is a gloo rehearsal of the multi-rank path on one GPU
            # (the ranks share it), not a scaling measurement
            "devices": min(world, ndev),
            "backend": (dist.get_backend() if world > 1 else None),
            "rehearsal": world > ndev,
            "roofline": {"bound": "mfma", "kernel": roof_name,
                         "achieved": round(achieved, 1) if achieved else None, "peak": peak, "unit": "TFLOP/s",
                         "frac": round(achieved / peak, 4) if achieved else None, "traffic": traffic,
                         "traffic_unit": "HBM bytes per launch (PMC FETCH_SIZE x2 + WRITE_SIZE)",
                         "traffic_source": traffic_src,
                         "algorithmic_bytes_per_launch": alg_bytes,
                         "flops_per_launch": fl_launch, "avg_launch_ms": round(avg_s * 1e3, 4), "launches": n1,
                         "rows_per_launch": round(rows_launch, 1),
                         "stream_split": enc.stream_split if n_chunks >= enc.split_min_chunks else 1,
                         # context, not the contract's peak: the bf16 MFMA rate this chip sustains on random
                         # operands (tools/mfma_peak.hip, 2 waves/SIMD, in-kernel clock 1.83 GHz) and the
                         # vendor GEMM on the same shape without bias/activation (tools/torch_gemm_ref.py)
                         "measured_mfma_ceiling": MEASURED_BF16_CEILING if args.dtype == "bf16" else None,
                         "frac_of_measured_ceiling": (round(achieved / MEASURED_BF16_CEILING, 4)
                                                      if achieved and args.dtype == "bf16" else None),
                         "hipblaslt_same_shape_tflops": HIPBLASLT_W1 if args.dtype == "bf16" else None,
                         # PMC: fraction of cycles the MFMA pipes were busy during this kernel, and the
                         # clock the chip held (GRBM_GUI_ACTIVE / 8 XCDs / duration), from the committed pass
                         "mfma_busy_pmc": busy if profiled else None,
                         "clock_ghz_pmc": busy_clk if profiled else None,
                         "mfma_busy_source": busy_src if profiled else None},
            "step_tflops_algorithmic": round(step_flops / (dt_max / args.steps) / 1e12, 1),
            "ctc_ms": round(ctc_ms, 3),
            "allgather_ids_ms": round(gather_ms, 3) if gather_ms is not None else None,
            "end_to_end_ms": round(e2e_ms, 3),
            "end_to_end_value": round(total_frames / (e2e_ms / 1e3), 1),
            "end_to_end_note": ("encoder step + fused CTC ids head" +
                                (" + ids all_gather_into_tensor and per-utterance reassembly" if world > 1 else "")),
            "allgather_logp_bf16_ms": round(gather_lp_ms, 3) if gather_lp_ms is not None else None,
            "reassembly_world8_ms": round(assemble_ms, 3) if assemble_ms is not None else None,
            "breakdown_ms": breakdown,
            "roofline_by_class": by_class,
        }
        if world == 1 and not args.no_cpu_baseline:
            res["cpu_baseline"] = cpu_baseline(lens_all)
        print(json.dumps(res), flush=True)
    if world > 1:
        dist.destroy_process_group()


def bench_single(args):
    """configs[3] (endless_decode, 16 h, one GPU) and configs[4] (full attention, B=256 x 30 s):
    one JSON line each, same keys as the headline line.  These run on one GPU only (configs[3] is
    sequential by construction; configs[4] is a parity / roofline check): --gpus must be 1."""
    from chunkformer_amd.model import ChunkFormerModel
    if args.gpus != 1:
        raise SystemExit(f"--config {args.config} runs on one GPU")
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    model = ChunkFormerModel(LARGE, synthetic_state_dict(LARGE, 0), dtype=args.dtype, device=dev)
    model.endless_fe_reuse = not args.no_fe_reuse
    if args.pipe_opt:
        from chunkformer_amd import streaming
        for kv in args.pipe_opt:
            k_, v_ = kv.split("=")
            streaming.PIPELINE_OPTS[k_] = int(v_)
    enc = model.encoder
    apply_opts(enc, args.opt)
    g = torch.Generator(device=dev).manual_seed(1234)
    d_, ff_ = LARGE.d_model, LARGE.ffn_dim
    if args.config == "endless":
        depth = args.pipeline_depth if args.pipeline_depth is not None else (3 if args.endless_mode == "pipeline" else 4)
        T = int(args.hours * 3600 * 100)
        x = torch.randn(T, 80, generator=g, device=dev)
        frames = T

        def step():
            return model.endless_decode(x, C, L, R, total_batch_duration=args.tbd, return_timestamps=False,
                                        pipeline=args.endless_mode in ("pipeline", "graphpipe"),
                                        cuda_graph=args.endless_mode != "pipeline", pipeline_depth=depth)
        from chunkformer_amd.model import endless_segments
        trunc, segs = endless_segments(T, C, L, R, args.tbd, LARGE.num_blocks, LARGE.kernel_size)
        seg_len = max(b - a for a, b, _, _ in segs)
        prof_x = [x[:seg_len]]
        prof_call = lambda: enc.forward_parallel_chunk(prof_x, torch.tensor([seg_len], dtype=torch.int32), C, L, R)
        rows = sum(chunks_of(seg_len, C) for _ in range(1)) * C
        roof_cls, attn_fl = "ffn_w1_gemm", None
        workload = (f"endless_decode over one {args.hours:g} h utterance (synthetic N(0,1) fbank), C=64 L=128 "
                    f"R=128, total_batch_duration={args.tbd}: {len(segs)} segments of <= {seg_len} frames "
                    f"(trunc {trunc} rows kept each), att/cnn caches carried, " +
                    {"graphpipe": f"{depth} segments in flight on as many HIP streams (segment k+1 "
                                  "layer l after segment k layer l), all segments (up to 128 per graph) one "
                                  "replay of a captured HIP graph of that whole multi-stream pipeline",
                     "pipeline": f"{depth} segments in flight on {depth} HIP streams "
                                 "(segment k+1 layer l waits for segment k layer l), launched eagerly",
                     "graph": "middle segments replayed one at a time from one captured HIP graph (front-end + "
                              "12 blocks + after_norm + CTC argmax)"}[args.endless_mode])
        extra = {"segments": len(segs), "segment_frames": seg_len, "truncated_context_size": trunc,
                 "fe_reuse": bool(model.endless_fe_reuse),
                 "pipeline_opts": dict(__import__("chunkformer_amd.streaming", fromlist=["x"]).PIPELINE_OPTS),
                 "endless_mode": args.endless_mode, "pipeline_depth": depth}
    else:
        B, T = args.batch, 3000
        xs = torch.randn(B, T, 80, generator=g, device=dev)
        lens = torch.full((B,), T, dtype=torch.int32)
        frames = B * T

        def step():
            return model.encode(xs, lens, -1, -1, -1)
        prof_call = step
        Tp = 1 + (T - 15) // 8
        rows = B * Tp
        roof_cls = "chunk_attention"
        # dense rel-pos attention per layer: scores T'xT', rel-pos band T'x(2T'-1), P.V T'xT' (x d, x2)
        attn_fl = 2.0 * B * Tp * d_ * (Tp + (2 * Tp - 1) + Tp)
        workload = (f"forward_encoder full attention (chunk_size=-1), B={B} x T={T} frames (30 s, T'={Tp}), "
                    f"synthetic N(0,1) fbank, padded batch")
        extra = {"batch": B, "frames_per_utt": T, "subsampled_frames": Tp}
    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    value = frames * args.steps / dt
    # roofline kernel: per-launch time from in-stream HIP events on an eager call of the same shape
    enc.set_option("profile_reset", 1)
    enc.set_option("profile", 1 << _lib.PROFILE_CLASSES.index(roof_cls))
    prof_call()
    torch.cuda.synchronize()
    enc.set_option("profile", 0)
    ms1, n1 = _lib.profile_read(enc._h)[roof_cls]
    avg_s = ms1 / max(n1, 1) / 1e3
    # per-class breakdown of one eager call (endless: one full segment)
    enc.set_option("profile_reset", 1)
    enc.set_option("profile", (1 << len(_lib.PROFILE_CLASSES)) - 1)
    prof_call()
    torch.cuda.synchronize()
    enc.set_option("profile", 0)
    breakdown = {k: round(v[0], 3) for k, v in _lib.profile_read(enc._h).items() if v[1]}
    peak = PEAK_TFLOPS[args.dtype]
    if roof_cls == "ffn_w1_gemm":
        fl_launch = 2.0 * rows * ff_ * d_
        kname = "ffn_w1_gemm (gemm_wsp_kernel<EPI_STORE,SiLU>: K=512 weight-stationary bf16 MFMA)"
    else:
        fl_launch = attn_fl
        kname = "chunk_attention (full_attention_bf16_kernel: every key of the utterance staged once per block)"
    achieved = fl_launch / avg_s / 1e12 if n1 else None
    res = {
        "metric": METRIC, "value": round(value, 1), "unit": "audio-frames/s", "n_gpus": 1, "steps": args.steps,
        "warmup": args.warmup, "ms_per_step": round(dt / args.steps * 1e3, 3), "higher_is_better": True,
        "scaling": "weak", "vs_baseline": None, "dtype": args.dtype,
        "data": "synthetic (N(0,1) 80-dim fbank, seeded random chunkformer-large weights; no checkpoint offline)",
        "config": {"workload": workload, "config_index": 3 if args.config == "endless" else 4, **extra,
                   "parallelism": "single GPU"},
        "roofline": {"bound": "mfma", "kernel": kname, "achieved": round(achieved, 1) if achieved else None,
                     "peak": peak, "unit": "TFLOP/s", "frac": round(achieved / peak, 4) if achieved else None,
                     "traffic": None, "flops_per_launch": fl_launch, "avg_launch_ms": round(avg_s * 1e3, 4),
                     "launches": n1},
        "breakdown_ms_one_call": breakdown,
    }
    print(json.dumps(res), flush=True)


def bench_fbank(args):
    """GPU Kaldi fbank (§8(f) row 2, chunkformer_model.py:306-314 parameters) over `--hours` of
    16 kHz int16-scale synthetic audio resident in HBM: frames/s, HBM roofline of the kernel
    (samples in + features out per launch), the CPU oracle (oracle/fbank_ref.py, torch float32,
    all cores) on 60 s of the same audio beside it."""
    from chunkformer_amd.fbank import KaldiFbank
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    n = int(args.hours * 3600 * 16000)
    g = torch.Generator(device=dev).manual_seed(7)
    x = (torch.randn(n, generator=g, device=dev) * 3000).round_()
    fb = KaldiFbank(dev, num_mel_bins=80, frame_length=25, frame_shift=10, dither=0.0, energy_floor=0.0,
                    sample_frequency=16000)
    frames = fb.num_frames(n)
    for _ in range(args.warmup):
        fb(x)
    torch.cuda.synchronize()
    st = torch.cuda.current_stream()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    t0 = time.perf_counter()
    e0.record(st)
    for _ in range(args.steps):
        fb(x)
    e1.record(st)
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    kern_s = e0.elapsed_time(e1) / 1e3 / args.steps
    nbytes = n * 4 + frames * 80 * 4
    from oracle import fbank_ref
    xs = x[: 60 * 16000].cpu()
    cpu_model, threads = host_cpu()
    torch.set_num_threads(threads)
    c0 = time.perf_counter()
    reps = 0
    while time.perf_counter() - c0 < 10.0:
        fbank_ref.fbank(xs, num_mel_bins=80, frame_length=25, frame_shift=10, dither=0.0, energy_floor=0.0)
        reps += 1
    cpu_fps = reps * fbank_ref.num_frames(xs.numel(), 400, 160) / (time.perf_counter() - c0)
    res = {
        "metric": "fbank frames/sec (80-dim Kaldi log-mel, 25/10 ms, povey) from 16 kHz audio resident in HBM",
        "value": round(frames * args.steps / dt, 1), "unit": "fbank-frames/s", "n_gpus": 1, "steps": args.steps,
        "warmup": args.warmup, "ms_per_step": round(dt / args.steps * 1e3, 3), "higher_is_better": True,
        "scaling": "weak", "vs_baseline": None, "dtype": "f32", "data": "synthetic (N(0, 3000^2) int16-scale samples)",
        "config": {"workload": f"kaldi.fbank over one {args.hours:g} h waveform ({n} samples, {frames} frames)",
                   "parallelism": "single GPU"},
        "roofline": {"bound": "hbm", "kernel": "fbank512_kernel (samples straight into registers, four-step 16x16 FFT, "
                                                "no block barriers, 3 blocks per CU)",
                     "achieved": round(nbytes / kern_s / 1e9, 1), "peak": 8000.0, "unit": "GB/s",
                     "frac": round(nbytes / kern_s / 1e9 / 8000.0, 4), "traffic": None,
                     "algorithmic_bytes_per_launch": nbytes, "avg_launch_ms": round(kern_s * 1e3, 3),
                     # the kernel's real bound is the vector ALU / LDS latency, not HBM: algorithmic FP32
                     # work per frame against the 157.3 TFLOP/s FP32 vector peak
                     "valu": {"flops_per_frame": FBANK_FLOPS_PER_FRAME,
                              "achieved_tflops": round(FBANK_FLOPS_PER_FRAME * frames / kern_s / 1e12, 2),
                              "peak_fp32_vector_tflops": 157.3,
                              "frac": round(FBANK_FLOPS_PER_FRAME * frames / kern_s / 1e12 / 157.3, 4)}},
        "cpu_baseline": {"value": round(cpu_fps, 1), "unit": "fbank-frames/s", "cores": threads, "cpu": cpu_model,
                         "kind": "port", "sample": "oracle/fbank_ref.py (torchaudio kaldi.fbank restated, torch "
                                                   "float32 CPU) on the first 60 s of the same audio, repeated ~10 s"},
    }
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
