"""Build an A/B variant of libcfm.so: the listed sources recompiled with extra -D flags, every
other object taken from chunkformer_amd/_build/ (build the product first).

    python tools/build_variant.py TAG gemm_wst.hip -DWSP_LGKM=0 [-DCFM_GEMM_DIAG ...]

writes chunkformer_amd/_build/variants/libcfm_TAG.so; select it with CFM_LIB=<path> (chunkformer_amd/_lib.py).
"""
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from chunkformer_amd import build as B  # noqa: E402


def main():
    tag, rest = sys.argv[1], sys.argv[2:]
    srcs = [a for a in rest if not a.startswith("-")]
    flags = [a for a in rest if a.startswith("-")]
    out = os.path.join(B.OUT, "variants")
    os.makedirs(out, exist_ok=True)
    objs = []
    for src in B._sources():
        name = os.path.basename(src)
        if name in srcs:
            obj = os.path.join(out, f"{name}.{tag}.o")
            cmd = [B.HIPCC, *B.FLAGS, *B.FILE_FLAGS.get(name, []), *flags, "-c", src, "-o", obj]
            r = subprocess.run(cmd, capture_output=True, text=True)
            if r.returncode:
                sys.exit(f"hipcc failed on {name}:\n{r.stderr}")
            objs.append(obj)
        else:
            objs.append(os.path.join(B.OUT, name + ".o"))
    lib = os.path.join(out, f"libcfm_{tag}.so")
    r = subprocess.run([B.HIPCC, f"--offload-arch={B.ARCH}", "-shared", "-fPIC", "-o", lib, *objs],
                       capture_output=True, text=True)
    if r.returncode:
        sys.exit(f"link failed:\n{r.stderr}")
    print(lib)


if __name__ == "__main__":
    main()
