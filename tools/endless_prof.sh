set -e
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/prof_endless
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 500 rocprofv3 --kernel-trace --stats --output-format csv -d $O/stats -o e -- python3 $R/bench.py --config endless --tbd 1800 --steps 1 --warmup 1 --no-cpu-baseline > $O/bench.log 2>&1
cp $(find $O/stats -name "*kernel_stats.csv" | head -1) $O/kernel_stats.csv
grep '^{' $O/bench.log | tail -1 | cut -c1-400
