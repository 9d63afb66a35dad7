# round 3: head_dim 128 attention kernel: parity + 4-head bench
set -e
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd $R
timeout -k 10 600 python3 -u -m pytest -x -v -s --timeout 300 --timeout-method thread "tests/test_gpu_scale.py::test_head_dim_128_kernel_vs_generic" "tests/test_gpu_scale.py::test_four_heads_head_dim_128" > gpurun_out/r3c.log 2>&1 || { tail -60 gpurun_out/r3c.log; exit 1; }
grep -E "PASS|FAIL|rel-L2" gpurun_out/r3c.log | tail -8
timeout -k 10 300 python3 bench.py --heads 4 --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/r3c_bench_4h.log 2>&1
grep '^{' gpurun_out/r3c_bench_4h.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], d['breakdown_ms'])"
