# A/B: weight-stationary GEMM barrier period 1 / 2 (product) / 4, then the full step
set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
VD=$GRAFT_REPO_ROOT/chunkformer_amd/_build/variants
for r in 1 2; do
  for v in bar1 prod bar4; do
    if [ $v = prod ]; then unset CFM_LIB; else export CFM_LIB=$VD/libcfm_$v.so; fi
    echo "== $v"; timeout -k 10 120 python3 tools/gemm_bench.py --iters 20 --only ffn_w1,qkv,out/pw2,pw1_glu,fe_pw1 2>&1 | grep -v amdgpu.ids
  done
done
unset CFM_LIB
CFM_LIB=$VD/libcfm_bar4.so timeout -k 10 300 python3 -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_ops.py 2>&1 | tail -1
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_ops.py tests/test_gpu_parity.py 2>&1 | tail -1
for v in bar1 prod bar4 prod; do
  if [ $v = prod ]; then unset CFM_LIB; else export CFM_LIB=$VD/libcfm_$v.so; fi
  timeout -k 10 300 python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/bar_b.json 2>/dev/null
  python3 -c "import json; d=json.loads(open('gpurun_out/bar_b.json').read().strip().splitlines()[-1]); print('$v', d['value'], d['ms_per_step'], d['roofline']['frac'])"
done
