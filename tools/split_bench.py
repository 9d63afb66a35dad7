"""Does running the configs[1] batch as S sub-batches on S streams (staggered by encoder layer via
cfm_encode_masked_stages) beat one launch sequence?  Timing only: the masked batch is per-utterance
independent, so the split changes no output.

    python tools/split_bench.py --parts 2 --rounds 3
"""
import argparse
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from bench import C, L, R, workload_lengths  # noqa: E402
from chunkformer_amd import _lib  # noqa: E402
from chunkformer_amd.config import LARGE  # noqa: E402
from chunkformer_amd.encoder import ChunkFormerEncoder  # noqa: E402
from chunkformer_amd.weights import synthetic_state_dict  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--parts", type=int, action="append", default=[])
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--minutes", type=float, default=240)
    a = ap.parse_args()
    parts_list = a.parts or [2]
    lens = workload_lengths(int(a.minutes * 6000), 0)
    g = torch.Generator(device="cuda").manual_seed(1)
    xs = [torch.randn(t, 80, generator=g, device="cuda") for t in lens]
    enc = ChunkFormerEncoder(LARGE, synthetic_state_dict(LARGE, 0), dtype="bf16")
    nb = LARGE.num_blocks
    xl = torch.tensor(lens, dtype=torch.int32)

    def prep(idx):
        ls = [lens[i] for i in idx]
        plan, n_chunks, _ = _lib.plan_masked(ls, [0] * len(ls), C, L, R)
        N = sum(n_chunks)
        feats = torch.cat([xs[i] for i in idx], 0).contiguous()
        wsb = int(_lib.cfm_workspace_bytes_masked(enc._h, N, C, L, R))
        return dict(plan=plan, plan_dev=enc._upload(plan), feats=feats, N=N, wsb=wsb,
                    ws=torch.empty(wsb, dtype=torch.uint8, device="cuda"),
                    out=torch.empty(N * C, LARGE.d_model, device="cuda"))

    def split(S):
        # utterances dealt round-robin by length (balanced chunk counts)
        order = sorted(range(len(lens)), key=lambda i: -lens[i])
        return [prep(order[s::S]) for s in range(S)]

    def call(p, lo, hi, st):
        _lib.check(_lib.cfm_encode_masked_stages(enc._h, p["feats"].data_ptr(), p["plan"].data_ptr(),
                                                 p["plan_dev"].data_ptr(), None, None, 0, None, None,
                                                 p["out"].data_ptr(), p["ws"].data_ptr(), p["wsb"], lo, hi, st))

    def run(parts, mode, streams):
        cur = torch.cuda.current_stream()
        if mode == "seq":
            for p in parts:
                call(p, -1, 1 << 30, cur.cuda_stream)
            return
        for s in streams:
            s.wait_stream(cur)
        prev = None
        for i, p in enumerate(parts):
            st = streams[i]
            evs = []
            for stage in range(-1, nb):
                if mode == "stag" and prev is not None and stage >= 0:
                    st.wait_event(prev[stage])
                call(p, stage, stage, st.cuda_stream)
                if mode == "stag":
                    e = torch.cuda.Event()
                    e.record(st)
                    evs.append(e)
            prev = evs
        for s in streams:
            cur.wait_stream(s)

    def timeit(fn):
        ts = []
        for r in range(a.rounds + 1):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            fn()
            torch.cuda.synchronize()
            if r:
                ts.append((time.perf_counter() - t0) * 1e3)
        return sorted(ts)[len(ts) // 2], min(ts)

    print("full batch, forward_parallel_chunk: median %.2f ms  min %.2f" % timeit(
        lambda: enc.forward_parallel_chunk(xs, xl, C, L, R)), flush=True)
    one = split(1)
    print("full batch, one stages call: median %.2f ms  min %.2f" % timeit(lambda: run(one, "seq", None)), flush=True)
    del one
    for S in parts_list:
        parts = split(S)
        streams = [torch.cuda.Stream() for _ in range(S)]
        for mode in ("seq", "stag", "free"):
            print(f"S={S} {mode}: median %.2f ms  min %.2f" % timeit(lambda: run(parts, mode, streams)), flush=True)
        del parts


if __name__ == "__main__":
    main()
