# front-end: linear/abs split of conv0+relu+dw1
set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python3 -u -m pytest -x -q -s --timeout 300 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_scale.py tests/test_gpu_model.py > gpurun_out/fe1.log 2>&1 || { tail -60 gpurun_out/fe1.log; exit 1; }
grep -E "golden utt|passed|failed" gpurun_out/fe1.log | tail -8
for i in 1 2; do
timeout -k 10 300 python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/fe1_b$i.json 2>/dev/null
python3 -c "import json; d=json.loads(open('gpurun_out/fe1_b$i.json').read().strip().splitlines()[-1]); b=d['breakdown_ms']; print(d['value'], d['ms_per_step'], {k: b[k] for k in b if k.startswith('frontend')})"
done
