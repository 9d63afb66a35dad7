# fused front-end pw1+dw2 (fe_fuse_dw2): bit-equality tests, then interleaved in-step A/B
set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 400 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_scale.py -k "fused_dw2" -s > gpurun_out/fuse_t.log 2>&1 || { tail -30 gpurun_out/fuse_t.log; exit 1; }
tail -5 gpurun_out/fuse_t.log
for v in 1 0 1 0; do
  timeout -k 10 300 python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline --opt fe_fuse_dw2=$v > gpurun_out/fuse_b.json 2>/dev/null
  python3 -c "import json; d=json.loads(open('gpurun_out/fuse_b.json').read().strip().splitlines()[-1]); b=d['breakdown_ms']; print('fuse=$v', d['value'], d['ms_per_step'], {k: b[k] for k in b if k.startswith('frontend')})"
done
