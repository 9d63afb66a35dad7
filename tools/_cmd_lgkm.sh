# in-step A/B: weight-stationary GEMM closing every K-step with lgkmcnt(0) (WSP_LGKM=0)
set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
VD=$GRAFT_REPO_ROOT/chunkformer_amd/_build/variants
for v in lgkm0 prod lgkm0 prod; do
  if [ $v = prod ]; then unset CFM_LIB; else export CFM_LIB=$VD/libcfm_$v.so; fi
  timeout -k 10 300 python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/lgkm_b.json 2>/dev/null
  python3 -c "import json; d=json.loads(open('gpurun_out/lgkm_b.json').read().strip().splitlines()[-1]); b=d['breakdown_ms']; print('$v', d['value'], d['ms_per_step'], b['ffn_w1_gemm'], b['qkv_gemm'])"
done
