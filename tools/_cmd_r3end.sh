# end-of-round check: full GPU suite + smoke on the final library, then the per-rank workload of the
# 8-way configs[2] split (122.5 min per GPU) and configs[2] on one GPU
set -e
cd $GRAFT_REPO_ROOT
bash tools/_cmd_suite.sh
timeout -k 10 300 python3 bench.py --minutes 122.5 --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/r3end_m122.log 2>&1
timeout -k 10 400 python3 bench.py --config sharded --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/r3end_cfg2_n1.log 2>&1
for f in r3end_m122 r3end_cfg2_n1; do grep '^{' gpurun_out/$f.log | tail -1 | cut -c1-400; done
