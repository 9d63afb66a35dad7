# in-step A/B at endless_decode's tbd-1800 segments: weight-stationary GEMM at any M (gemm_wst=2)
set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for o in gemm_wst=1 gemm_wst=2 gemm_wst=1 gemm_wst=2; do
  timeout -k 10 300 python3 bench.py --config endless --tbd 1800 --steps 2 --warmup 1 --no-cpu-baseline --opt $o > gpurun_out/endwst.json 2>/dev/null
  python3 -c "import json; d=json.loads(open('gpurun_out/endwst.json').read().strip().splitlines()[-1]); print('$o', d['value'], d['ms_per_step'])"
done
