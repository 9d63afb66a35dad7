# in-step A/B: 256 x 256 GEMM wave priorities
set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
VD=$GRAFT_REPO_ROOT/chunkformer_amd/_build/variants
for v in prod p5 p6 prod p5 p6; do
  if [ $v = prod ]; then unset CFM_LIB; else export CFM_LIB=$VD/libcfm_$v.so; fi
  timeout -k 10 300 python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/prio_b.json 2>/dev/null
  python3 -c "import json; d=json.loads(open('gpurun_out/prio_b.json').read().strip().splitlines()[-1]); b=d['breakdown_ms']; print('$v', d['value'], d['ms_per_step'], b['ffn_w2_gemm'])"
done
