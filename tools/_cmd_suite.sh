# full GPU suite + smoke
set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -v -s --timeout 300 --timeout-method thread > gpurun_out/suite.log 2>&1 || { tail -40 gpurun_out/suite.log; exit 1; }
grep -E "golden utt|passed|failed" gpurun_out/suite.log | tail -6
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" 2>&1 | grep -v amdgpu.ids | tail -3
