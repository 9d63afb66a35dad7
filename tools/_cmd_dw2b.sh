# dw2 with packed input rows (4 waves/SIMD): parity + in-step timing
set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_scale.py tests/test_gpu_model.py 2>&1 | tail -1
for i in 1 2 3; do
  timeout -k 10 300 python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/dw2b.json 2>/dev/null
  python3 -c "import json; d=json.loads(open('gpurun_out/dw2b.json').read().strip().splitlines()[-1]); b=d['breakdown_ms']; print(d['value'], d['ms_per_step'], b['frontend_dw2'], b['conv_dw_ln_silu'])"
done
