# fused pw1+dw2: store-policy / barrier-period / deferred-store A/B in the step (frontend pw breakdown)
set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
VD=$GRAFT_REPO_ROOT/chunkformer_amd/_build/variants
CFM_LIB=$VD/libcfm_dwdf.so timeout -k 10 300 python3 -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_scale.py -k "fused_dw2" > gpurun_out/dw2st_t.log 2>&1 || { tail -30 gpurun_out/dw2st_t.log; exit 1; }
tail -1 gpurun_out/dw2st_t.log
for v in prod b1 nt df dfnt prod b1 nt df dfnt; do
  case $v in prod) unset CFM_LIB;; *) export CFM_LIB=$VD/libcfm_dw$v.so;; esac
  timeout -k 10 300 python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/dw2st_b.json 2>/dev/null
  python3 -c "import json; d=json.loads(open('gpurun_out/dw2st_b.json').read().strip().splitlines()[-1]); b=d['breakdown_ms']; print('$v', d['value'], d['ms_per_step'], {k: b[k] for k in b if k.startswith('frontend')})" | tee -a gpurun_out/dw2st_ab.txt
done
