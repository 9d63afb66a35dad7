# full GPU suite + smoke (the driver's round-end check)
set -e
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd $R
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/full.log 2>&1 || { tail -40 gpurun_out/full.log; exit 1; }
tail -3 gpurun_out/full.log
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" 2>&1 | tail -2
