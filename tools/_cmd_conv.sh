# in-step A/B: conv module depthwise via dot2 (default) vs the per-tap f32 kernel
set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for o in conv_dot2=1 conv_dot2=2 conv_dot2=1 conv_dot2=2; do
  timeout -k 10 300 python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline --opt $o > gpurun_out/conv_b.json 2>/dev/null
  python3 -c "import json; d=json.loads(open('gpurun_out/conv_b.json').read().strip().splitlines()[-1]); b=d['breakdown_ms']; print('$o', d['value'], d['ms_per_step'], b['conv_dw_ln_silu'], b['pw2_gemm'])"
done
