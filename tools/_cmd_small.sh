# per-rank batch of configs[2] at N = 8 (980/8 min): plain vs stream_split=2
set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for o in stream_split=1 stream_split=2 stream_split=1 stream_split=2; do
  timeout -k 10 300 python3 bench.py --config masked --minutes 122.5 --steps 10 --warmup 2 --no-cpu-baseline --no-breakdown --opt $o > gpurun_out/small_b.json 2>/dev/null
  python3 -c "import json; d=json.loads(open('gpurun_out/small_b.json').read().strip().splitlines()[-1]); print('$o', d['value'], d['ms_per_step'], d['config']['chunks_rank0'], d['roofline']['frac'])"
done
