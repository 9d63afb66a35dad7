"""Per-kernel HBM traffic per launch from rocprofv3 PMC passes (MI355X_MICROARCH.md, HBM
section): FETCH_SIZE and WRITE_SIZE are collected in SEPARATE passes (TCC slots), both in
KiB; on gfx950 FETCH_SIZE reports half the bytes of wide coalesced streaming reads, so it
is doubled.  Writes `profiles/<round>_traffic.json`:

    python tools/traffic.py FETCH_DIR WRITE_DIR OUT_JSON
"""
import csv
import glob
import json
import sys
from collections import defaultdict

# kernel-name fragment -> libcfm profiler class (model.hip PROF classes)
CLASSES = [
    ("gemm_bf16_256_kernel<0, 2,", "ffn_w1_gemm"), ("gemm_bf16_256_kernelILi0ELi2E", "ffn_w1_gemm"),
    ("gemm_bf16_256_kernel<2, 0,", "resid_gemm (ffn_w2 / out_proj / pw2)"),
    ("gemm_bf16_256_kernel<3, 0,", "qkv_gemm"), ("gemm_bf16_256_kernel<4, 0,", "pw1_glu_gemm"),
    ("gemm_bf16_256_kernel<0, 1,", "frontend_pw_gemm"),
    ("gemm_bf16_256_kernel<0, 0,", "plain_gemm_k2048+ (ffn_w2 / frontend out)"),
    ("gemm_wsp_kernel<0, 2,", "ffn_w1_gemm"), ("gemm_wsp_kernelILi0ELi2E", "ffn_w1_gemm"),
    # ACT_SILU_L2E (3): the 16-bit modes' FFN w1 and (with EPI_GLU = 4) the conv module's pw1
    ("gemm_wsp_kernel<0, 3,", "ffn_w1_gemm"), ("gemm_wsp_kernelILi0ELi3E", "ffn_w1_gemm"),
    ("gemm_bf16_256_kernel<0, 3,", "ffn_w1_gemm"), ("gemm_bf16_256_kernelILi0ELi3E", "ffn_w1_gemm"),
    ("gemm_wsp_kernel<4, 3,", "pw1_glu_gemm"), ("gemm_bf16_256_kernel<4, 3,", "pw1_glu_gemm"),
    ("gemm_wsp_kernel<5, 1,", "frontend_pw1_dw2 (fused)"), ("gemm_wsp_kernelILi5ELi1E", "frontend_pw1_dw2 (fused)"),
    ("gemm_wsp_kernel<0, 1,", "frontend_pw_gemm"), ("gemm_wsp_kernel<3, 0,", "qkv_gemm"),
    ("gemm_wsp_kernel<4, 0,", "pw1_glu_gemm"), ("gemm_wsp_kernel<0, 0,", "plain_gemm_k512 (out_proj / pw2)"),
    ("fe_conv0_dw_mfma2_kernel", "frontend_conv0_dw"),
    ("fe_conv0_dw_mfma_kernel", "frontend_conv0_dw"),
    ("fe_dw2_kernel", "frontend_dw2"),
    ("chunk_attention_ring_kernel", "chunk_attention"),
    ("conv_dw_ln_silu", "conv_dw_ln_silu"),
    ("ln_kernel", "layernorm"),
    ("ln2_kernel", "layernorm2"),
]


def per_dispatch(d, counter):
    tot, n = defaultdict(float), defaultdict(set)
    for f in glob.glob(f"{d}/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            if r["Counter_Name"] != counter:
                continue
            k = r["Kernel_Name"]
            tot[k] += float(r["Counter_Value"])
            n[k].add(r["Dispatch_Id"])
    return {k: (tot[k] / len(n[k]), len(n[k])) for k in tot}


def main():
    fd, wd, out = sys.argv[1:4]
    fetch, write = per_dispatch(fd, "FETCH_SIZE"), per_dispatch(wd, "WRITE_SIZE")
    res = {}
    for k in sorted(set(fetch) | set(write)):
        cls = next((c for frag, c in CLASSES if frag in k), None)
        if cls is None:
            continue
        f_kib, nf = fetch.get(k, (0.0, 0))
        w_kib, nw = write.get(k, (0.0, 0))
        res.setdefault(cls, []).append({
            "kernel": k[:120], "dispatches": max(nf, nw),
            "fetch_bytes_per_launch": 2.0 * f_kib * 1024, "write_bytes_per_launch": w_kib * 1024,
            "hbm_bytes_per_launch": 2.0 * f_kib * 1024 + w_kib * 1024})
    json.dump({"note": "rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE in separate passes; FETCH x2 (gfx950 correction)",
               "kernels": res}, open(out, "w"), indent=1)
    for c, v in res.items():
        for e in v:
            print(f"{c:20s} {e['hbm_bytes_per_launch'] / 1e9:10.3f} GB/launch  n={e['dispatches']}  {e['kernel'][:60]}")


if __name__ == "__main__":
    main()
