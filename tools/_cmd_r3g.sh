# round 3: masked batch as utterance groups on staggered streams
set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread "tests/test_gpu_scale.py::test_stream_split_bit_identical" "tests/test_gpu_scale.py::test_golden_utterances_inside_bench_batch" tests/test_gpu_sharded.py > gpurun_out/r3g.log 2>&1 || { tail -60 gpurun_out/r3g.log; exit 1; }
tail -12 gpurun_out/r3g.log
for sp in 2 1 2 1; do
  timeout -k 10 300 python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline --opt stream_split=$sp > gpurun_out/r3g_b$sp.json 2>/dev/null
  python3 -c "import json; d=json.loads(open('gpurun_out/r3g_b$sp.json').read().strip().splitlines()[-1]); r=d['roofline']; print($sp, d['value'], d['ms_per_step'], d['end_to_end_ms'], r['frac'], r['avg_launch_ms'], r['launches'], r['rows_per_launch'])"
done
