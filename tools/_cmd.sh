# Round check on one GPU (run via gpurun from the repo root): GPU parity tests, smoke, bf16 accuracy
# probe and the default bench line.
set -e
cd $GRAFT_REPO_ROOT
timeout -k 10 600 python3 -u -m pytest tests/ -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || { tail -30 gpurun_out/gpu_tests.log; exit 1; }
tail -1 gpurun_out/gpu_tests.log
timeout -k 10 120 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { tail -20 gpurun_out/smoke.log; exit 1; }
tail -1 gpurun_out/smoke.log
timeout -k 10 120 python3 tools/bf16_err.py > gpurun_out/bf16_err.log 2>&1 || { tail -20 gpurun_out/bf16_err.log; exit 1; }
grep "rel-L2" gpurun_out/bf16_err.log
timeout -k 10 300 python3 bench.py > gpurun_out/bench.log 2>&1 || { tail -20 gpurun_out/bench.log; exit 1; }
tail -1 gpurun_out/bench.log
