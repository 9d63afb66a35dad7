# round 3: RNN-T consumer, checkpoint CMVN, rows != origin lens
set -e
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd $R
timeout -k 10 900 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_rnnt.py tests/test_gpu_checkpoint.py "tests/test_gpu_parity.py::test_rows_differ_from_origin_lens" > gpurun_out/r3b.log 2>&1 || { tail -60 gpurun_out/r3b.log; exit 1; }
tail -15 gpurun_out/r3b.log
timeout -k 10 300 python3 bench.py --heads 4 --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/r3b_bench_4h.log 2>&1
grep '^{' gpurun_out/r3b_bench_4h.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], d['breakdown_ms'])"
