# 256 x 256 GEMM with 32-deep K-steps: numerics, microbench A/B, bench A/B
set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_ops.py > gpurun_out/k32.log 2>&1 || { tail -30 gpurun_out/k32.log; exit 1; }
tail -1 gpurun_out/k32.log
for r in 1 2; do
  for k in 2 1; do
    echo "== k32=$k"; timeout -k 10 120 python3 tools/gemm_bench.py --iters 20 --only ffn_w2 --k32 $k 2>&1 | grep -v amdgpu.ids
  done
done
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_scale.py > gpurun_out/k32b.log 2>&1 || { tail -30 gpurun_out/k32b.log; exit 1; }
tail -1 gpurun_out/k32b.log
for k in 0 1 0 1; do
  timeout -k 10 300 python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline --opt gemm_k32=$k > gpurun_out/k32_b.json 2>/dev/null
  python3 -c "import json; d=json.loads(open('gpurun_out/k32_b.json').read().strip().splitlines()[-1]); b=d['breakdown_ms']; print('k32=$k', d['value'], d['ms_per_step'], b['ffn_w2_gemm'], b['frontend_pw_gemm'])"
done
