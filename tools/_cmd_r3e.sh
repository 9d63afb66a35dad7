# round 3: endless_decode with two segments in flight (configs[3] at tbd 1800 and 7200)
set -e
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd $R
timeout -k 10 600 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread "tests/test_gpu_model.py::test_endless_graph_replay_equals_eager" "tests/test_gpu_scale.py::test_large_endless_decode" tests/test_gpu_rnnt.py > gpurun_out/r3e.log 2>&1 || { tail -60 gpurun_out/r3e.log; exit 1; }
tail -12 gpurun_out/r3e.log
for mode in pipeline graph; do
  for tbd in 1800 7200; do
    timeout -k 10 300 python3 bench.py --config endless --tbd $tbd --endless-mode $mode --steps 2 --warmup 1 > gpurun_out/r3e_${mode}_${tbd}.json 2>gpurun_out/r3e_${mode}_${tbd}.err
    python3 -c "import json; d=json.loads(open('gpurun_out/r3e_${mode}_${tbd}.json').read().strip().splitlines()[-1]); print('$mode', $tbd, d['value'], d['ms_per_step'])"
  done
done
