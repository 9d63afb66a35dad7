# conv module: GPU suite on the half-chunk default, then in-step A/B of 1 / 2 / 3 (whole / half / quarter chunks)
set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/suite2.log 2>&1 || { tail -30 gpurun_out/suite2.log; exit 1; }
tail -1 gpurun_out/suite2.log
for o in conv_dot2=1 conv_dot2=2 conv_dot2=3 conv_dot2=2 conv_dot2=3; do
  timeout -k 10 300 python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline --opt $o > gpurun_out/conv_b.json 2>/dev/null
  python3 -c "import json; d=json.loads(open('gpurun_out/conv_b.json').read().strip().splitlines()[-1]); b=d['breakdown_ms']; print('$o', d['value'], d['ms_per_step'], b['conv_dw_ln_silu'])"
done
