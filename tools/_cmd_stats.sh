# kernel-trace stats of the default bench (one GPU); summary -> gpurun_out/stats/kernel_stats.csv
set -e
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/stats
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/raw -o bench -- python3 $R/bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-breakdown > $O/stats_bench.log 2>&1
cp $(find $O/raw -name "*kernel_stats.csv" | head -1) $O/kernel_stats.csv
rm -rf $O/raw
