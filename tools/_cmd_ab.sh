# in-process A/B of model options (tools/ab_bench.py); args passed through
set -e
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd $R
timeout -k 10 400 python3 tools/ab_bench.py "$@" > gpurun_out/ab.log 2>&1 || { tail -30 gpurun_out/ab.log; exit 1; }
cat gpurun_out/ab.log | grep -v amdgpu.ids
