# fused front-end pw1+dw2: bit-equality of the product build, then in-step A/B of dw2-phase variants
set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 400 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_scale.py -k "fused_dw2" > gpurun_out/fuse_t.log 2>&1 || { tail -30 gpurun_out/fuse_t.log; exit 1; }
tail -3 gpurun_out/fuse_t.log
timeout -k 10 200 python3 tools/large12_err.py | tee gpurun_out/large12_err.txt
VD=$GRAFT_REPO_ROOT/chunkformer_amd/_build/variants
for v in prod0 prod p2 nost noph prod0 prod p2 prod0 prod; do
  opt="--opt fe_fuse_dw2=1"
  case $v in prod) unset CFM_LIB;; prod0) unset CFM_LIB; opt="--opt fe_fuse_dw2=0";; *) export CFM_LIB=$VD/libcfm_dw$v.so;; esac
  timeout -k 10 300 python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline $opt > gpurun_out/fuse_b.json 2>/dev/null
  python3 -c "import json; d=json.loads(open('gpurun_out/fuse_b.json').read().strip().splitlines()[-1]); b=d['breakdown_ms']; print('$v', d['value'], d['ms_per_step'], {k: b[k] for k in b if k.startswith('frontend')})" | tee -a gpurun_out/fuse_ab.txt
done
