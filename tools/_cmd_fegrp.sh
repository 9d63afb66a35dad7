# front-end window-group size sweep (MALL residency of the intermediates)
set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for g in 0 32 64 96 128 192; do
  timeout -k 10 300 python3 bench.py --steps 8 --warmup 2 --no-cpu-baseline --opt fe_group_windows=$g > gpurun_out/fegrp_$g.json 2>/dev/null
  python3 -c "import json; d=json.loads(open('gpurun_out/fegrp_$g.json').read().strip().splitlines()[-1]); b=d['breakdown_ms']; print($g, d['value'], d['ms_per_step'], {k: b[k] for k in b if k.startswith('frontend')}, round(sum(b[k] for k in b if k.startswith('frontend')),3))"
done
