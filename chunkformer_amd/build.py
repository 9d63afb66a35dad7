"""Build libcfm.so (gfx950) from chunkformer_amd/csrc with hipcc, in-tree.

    python -m chunkformer_amd.build          # incremental
    python -m chunkformer_amd.build --force

Objects and the library land in chunkformer_amd/_build/ (git-ignored, but they
travel to the GPU box with the gpurun snapshot).
"""
from __future__ import annotations

import concurrent.futures as cf
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(HERE, "csrc")
OUT = os.path.join(HERE, "_build")
LIB = os.path.join(OUT, "libcfm.so")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
ARCH = os.environ.get("CFM_ARCH", "gfx950")
FLAGS = ["-O3", "-std=c++17", "-fPIC", f"--offload-arch={ARCH}", "-Wno-unused-result"]
# frontend.hip: ReLU on MFMA outputs as a single v_max_f32 (no IEEE-mode canonicalisation);
# the front-end never sees NaN inputs it would have to propagate; no SLP packing of the ReLU.w1
# FMAs into v_pk_fma_f32 (slower issue beside MFMAs)
FILE_FLAGS = {"frontend.hip": ["-fno-honor-nans", "-mno-amdgpu-ieee", "-fno-slp-vectorize"]}


def _sources():
    return sorted(os.path.join(CSRC, f) for f in os.listdir(CSRC) if f.endswith((".hip", ".cpp")))


def _headers():
    hs = [os.path.join(CSRC, f) for f in os.listdir(CSRC) if f.endswith(".h")]
    hs.append(os.path.join(os.path.dirname(HERE), "include", "cfm.h"))
    return hs


def _compile(src: str, force: bool) -> str:
    obj = os.path.join(OUT, os.path.basename(src) + ".o")
    newest_dep = max(os.path.getmtime(p) for p in [src] + _headers())
    if not force and os.path.exists(obj) and os.path.getmtime(obj) >= newest_dep:
        return obj
    cmd = [HIPCC, *FLAGS, *FILE_FLAGS.get(os.path.basename(src), []), "-c", src, "-o", obj]
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"hipcc failed on {src}:\n{r.stdout}\n{r.stderr}")
    return obj


def build(force: bool = False, jobs: int = 8) -> str:
    os.makedirs(OUT, exist_ok=True)
    # the weight-stationary GEMM's translation units take minutes each (heavily unrolled kernels): start
    # them first so that the parallel build ends with the short ones
    srcs = sorted(_sources(), key=lambda p: (0 if "gemm_wst_" in os.path.basename(p) else 1, -os.path.getsize(p)))
    with cf.ThreadPoolExecutor(max_workers=jobs) as ex:
        objs = list(ex.map(lambda s: _compile(s, force), srcs))
    if force or not os.path.exists(LIB) or os.path.getmtime(LIB) < max(os.path.getmtime(o) for o in objs):
        cmd = [HIPCC, f"--offload-arch={ARCH}", "-shared", "-fPIC", "-o", LIB, *objs]
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError(f"link failed:\n{r.stdout}\n{r.stderr}")
    return LIB


if __name__ == "__main__":
    print(build(force="--force" in sys.argv))
