# per-kernel rocprof averages of one bench config for several libraries, interleaved
# usage: VARIANTS="base dnoovl base2 dnoovlb" BCFG=full KERNEL=full_attention bash tools/ab_kstats.sh
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out; mkdir -p $O
for v in ${VARIANTS}; do
  L=chunkformer_amd/_build/libcfm.so; case $v in base*) ;; *) L=chunkformer_amd/_build/variants/libcfm_${v%b}.so;; esac
  CFM_LIB=$PWD/$L timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/ks_$v -o ks -- python3 bench.py --config ${BCFG:-masked} --no-cpu-baseline --no-breakdown --steps 10 > $O/ks_$v.log 2>&1
  f=$(find $O/ks_$v -name '*kernel_stats.csv' | head -1)
  python3 - "$f" "$v" <<'PY'
import csv, os, sys
k = os.environ.get("KERNEL", "chunk_attention")
for r in csv.DictReader(open(sys.argv[1])):
    if k in r["Name"]:
        print(sys.argv[2], r["Name"][:60], r["Calls"], "avg %.1f us" % (float(r["AverageNs"]) / 1e3))
PY
done
