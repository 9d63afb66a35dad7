# round 3: configs[2] world-8 test + sharded tests, then the 2-rank rehearsal through bench --gpus 2
set -e
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd $R
timeout -k 10 600 python3 -u -m pytest -x -v -s --timeout 300 --timeout-method thread tests/test_gpu_sharded.py > gpurun_out/r3a_sharded.log 2>&1
tail -5 gpurun_out/r3a_sharded.log
grep "configs\[2\] world 8" gpurun_out/r3a_sharded.log || true
bash tools/_cmd_rehearse.sh
