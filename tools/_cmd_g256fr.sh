# A/B in the step: 256 x 256 GEMM EPI_STORE epilogue as full-row stores (product) vs 64-B pieces (fr0)
set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
VD=$GRAFT_REPO_ROOT/chunkformer_amd/_build/variants
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_ops.py 2>&1 | tail -1
for v in fr0 prod fr0 prod fr0 prod; do
  if [ $v = prod ]; then unset CFM_LIB; else export CFM_LIB=$VD/libcfm_$v.so; fi
  timeout -k 10 300 python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/g256_b.json 2>/dev/null
  python3 -c "import json; d=json.loads(open('gpurun_out/g256_b.json').read().strip().splitlines()[-1]); b=d['breakdown_ms']; print('$v', d['value'], d['ms_per_step'], b['ffn_w2_gemm'], b['frontend_pw_gemm'])"
done
