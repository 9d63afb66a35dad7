"""Which half of streaming.destroy_graphs' ordering the round-5 replay segfault needed.

    python tools/graph_destroy_probe.py nosync     # destroy graphs without the device sync (events kept)
    python tools/graph_destroy_probe.py early_ev   # sync, but release the capture events before the graphs
    python tools/graph_destroy_probe.py both       # neither
    python tools/graph_destroy_probe.py temp_events   # round 4's capture: the events recorded inside a capture
                                                      # are not kept (released while the capture still runs)

Each variant monkeypatches streaming.destroy_graphs and then runs tools/endless_seq.py's sequence (three
models, every endless mode, runners replaced between them) in this process; a segfault ends the process.
Run one variant per process (and one process per gpurun call after a fault)."""
import faulthandler
import gc
import os
import sys

import torch

faulthandler.enable()
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tools"))
from chunkformer_amd import streaming  # noqa: E402


def make(variant):
    def destroy(entries, device):
        entries = [e for e in entries if e is not None]
        if not entries:
            return
        if variant == "early_ev":
            torch.cuda.synchronize(device)
        for e in entries:
            if isinstance(e, tuple) and variant in ("early_ev", "both"):
                e[1].clear()   # the events recorded in the capture go first
                gc.collect()
            (e[0] if isinstance(e, tuple) else e).reset()
    return destroy


def main():
    variant = sys.argv[1]
    assert variant in ("nosync", "early_ev", "both", "temp_events")
    if variant == "temp_events":
        import inspect
        import textwrap
        src = textwrap.dedent(inspect.getsource(streaming.EndlessGraphPipeline._run))
        src = src.replace("keep.append(e)", "pass").replace("keep.extend(gp)", "pass")
        ns = {}
        exec(compile(src, streaming.__file__, "exec"), vars(streaming), ns)
        streaming.EndlessGraphPipeline._run = ns["_run"]
    else:
        streaming.destroy_graphs = make(variant)
    import endless_seq
    sys.argv = [sys.argv[0], "m32,mb,m16,g32,gb,g16,g32,gb"]
    endless_seq.main()
    print("variant", variant, "survived", flush=True)


if __name__ == "__main__":
    main()
