set -e
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 python3 $R/bench.py --config fbank --steps 5 --warmup 1 > $R/gpurun_out/fbank_bench.log 2>&1
tail -1 $R/gpurun_out/fbank_bench.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/fbank_prof -o fb -- python3 $R/bench.py --config fbank --steps 3 --warmup 1 > $R/gpurun_out/fbank_prof.log 2>&1
grep fbank $R/gpurun_out/fbank_prof/*/fb_kernel_stats.csv $R/gpurun_out/fbank_prof/fb_kernel_stats.csv 2>/dev/null | cut -c1-200 || true
