# A/B: front-end dw2 with non-temporal input loads; dw2_seg sweep
set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
VD=$GRAFT_REPO_ROOT/chunkformer_amd/_build/variants
for v in prod dw2nt prod dw2nt; do
  if [ $v = prod ]; then unset CFM_LIB; else export CFM_LIB=$VD/libcfm_$v.so; fi
  timeout -k 10 300 python3 bench.py --steps 8 --warmup 2 --no-cpu-baseline > gpurun_out/dw2_b.json 2>/dev/null
  python3 -c "import json; d=json.loads(open('gpurun_out/dw2_b.json').read().strip().splitlines()[-1]); b=d['breakdown_ms']; print('$v', d['value'], d['ms_per_step'], b['frontend_dw2'], b['frontend_pw_gemm'])"
done
unset CFM_LIB
for sg in 2 3 6 8; do
  timeout -k 10 300 python3 bench.py --steps 8 --warmup 2 --no-cpu-baseline --opt dw2_seg=$sg > gpurun_out/dw2_b.json 2>/dev/null
  python3 -c "import json; d=json.loads(open('gpurun_out/dw2_b.json').read().strip().splitlines()[-1]); b=d['breakdown_ms']; print('seg $sg', d['value'], d['ms_per_step'], b['frontend_dw2'])"
done
