# Bench lines of the non-default configs on one GPU (run via gpurun from the repo root):
# configs[3] endless, configs[4] full attention, configs[2] sharded batch at world size 1, fbank.
set -e
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/configs; mkdir -p $O
timeout -k 10 400 python3 $R/bench.py --config endless --steps 2 --warmup 1 > $O/endless.log 2>&1
tail -1 $O/endless.log
timeout -k 10 300 python3 $R/bench.py --config full --steps 3 --warmup 1 > $O/full.log 2>&1
tail -1 $O/full.log
timeout -k 10 400 python3 $R/bench.py --config sharded --steps 2 --warmup 1 --no-cpu-baseline > $O/sharded.log 2>&1
tail -1 $O/sharded.log
timeout -k 10 300 python3 $R/bench.py --config fbank --steps 5 --warmup 1 > $O/fbank.log 2>&1
tail -1 $O/fbank.log
