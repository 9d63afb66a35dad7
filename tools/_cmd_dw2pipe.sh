# fused pw1+dw2: software-pipelined dw2 taps (DW2_PIPE) -- bit-identity, then in-step A/B
set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
VD=$GRAFT_REPO_ROOT/chunkformer_amd/_build/variants
for v in pipe pipe2; do
  CFM_LIB=$VD/libcfm_dw$v.so timeout -k 10 300 python3 -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_scale.py -k "fused_dw2" > gpurun_out/dw2pipe_t.log 2>&1 || { tail -30 gpurun_out/dw2pipe_t.log; exit 1; }
  tail -1 gpurun_out/dw2pipe_t.log
done
for v in prod pipe pipe2 prod pipe pipe2 prod pipe pipe2; do
  case $v in prod) unset CFM_LIB;; *) export CFM_LIB=$VD/libcfm_dw$v.so;; esac
  timeout -k 10 300 python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/dw2pipe_b.json 2>/dev/null
  python3 -c "import json; d=json.loads(open('gpurun_out/dw2pipe_b.json').read().strip().splitlines()[-1]); b=d['breakdown_ms']; print('$v', d['value'], d['ms_per_step'], {k: b[k] for k in b if k.startswith('frontend')})" | tee -a gpurun_out/dw2pipe_ab.txt
done
