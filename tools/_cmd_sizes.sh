# per-class time per chunk at 240 min vs 122.5 min (the per-rank share of configs[2] at N = 8)
set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for m in 240 122.5; do
  timeout -k 10 300 python3 bench.py --minutes $m --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/sz_$m.json 2>/dev/null
  python3 -c "
import json; d=json.loads(open('gpurun_out/sz_$m.json').read().strip().splitlines()[-1]); n=d['config']['chunks_rank0']; b=d['breakdown_ms']
print('$m', n, d['value'], d['ms_per_step'], round(sum(b.values()),2))
print({k: round(v/n*1000, 2) for k, v in b.items()})"
done
