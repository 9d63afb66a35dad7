# round 3: endless pipeline depth sweep at tbd 1800 / 7200
set -e
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd $R
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 200 --timeout-method thread "tests/test_gpu_model.py::test_endless_graph_replay_equals_eager" > gpurun_out/r3f.log 2>&1 || { tail -60 gpurun_out/r3f.log; exit 1; }
tail -2 gpurun_out/r3f.log
for tbd in 1800 7200; do
  for dp in 2 3 4; do
    timeout -k 10 300 python3 bench.py --config endless --tbd $tbd --pipeline-depth $dp --steps 3 --warmup 1 > gpurun_out/r3f_${dp}_${tbd}.json 2>gpurun_out/r3f_${dp}_${tbd}.err
    python3 -c "import json; d=json.loads(open('gpurun_out/r3f_${dp}_${tbd}.json').read().strip().splitlines()[-1]); print($dp, $tbd, d['value'], d['ms_per_step'])"
  done
done
