# Round profile on ONE GPU (run via gpurun from the repo root):
#   kernel-trace stats of the bench, PMC HBM traffic (FETCH / WRITE in separate passes),
#   then the plain bench line.  Summaries land in gpurun_out/prof_<round>/; copy them to
#   profiles/<round>_* (traffic.json, mfma_busy.json, kernel_stats.csv, bench.json) afterwards.
set -e
RND=${1:-r02}
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/prof_$RND
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
if [ "$2" != "pmc" ]; then
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/stats -o bench -- python3 $R/bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-breakdown > $O/stats_bench.log 2>&1
fi
timeout -k 10 400 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/fetch -o f -- python3 $R/bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-breakdown > $O/fetch.log 2>&1
timeout -k 10 400 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/write -o w -- python3 $R/bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-breakdown > $O/write.log 2>&1
python3 $R/tools/traffic.py $O/fetch $O/write $O/traffic.json > $O/traffic.txt
timeout -k 10 400 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES --output-format csv -d $O/mfma -o m -- python3 $R/bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-breakdown > $O/mfma.log 2>&1
python3 $R/tools/mfma_busy.py $O/mfma $O/mfma_busy.json > $O/mfma_busy.txt
if [ "$2" != "pmc" ]; then
cp $(find $O/stats -name "*kernel_stats.csv" | head -1) $O/kernel_stats.csv
timeout -k 10 400 python3 $R/bench.py > $O/bench.log 2>&1
tail -1 $O/bench.log > $O/bench.json
fi
