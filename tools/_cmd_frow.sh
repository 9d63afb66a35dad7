# A/B in the real step: full-row stores also for the SiLU / ReLU epilogues (WSP_FULLROW_ACT=1)
set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
VD=$GRAFT_REPO_ROOT/chunkformer_amd/_build/variants
CFM_LIB=$VD/libcfm_frow.so timeout -k 10 300 python3 -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_ops.py 2>&1 | tail -1
for v in prod frow prod frow prod frow; do
  if [ $v = prod ]; then unset CFM_LIB; else export CFM_LIB=$VD/libcfm_$v.so; fi
  timeout -k 10 300 python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/frow_b.json 2>/dev/null
  python3 -c "import json; d=json.loads(open('gpurun_out/frow_b.json').read().strip().splitlines()[-1]); b=d['breakdown_ms']; print('$v', d['value'], d['ms_per_step'], d['roofline']['frac'], b['ffn_w1_gemm'], b['frontend_pw_gemm'])"
done
