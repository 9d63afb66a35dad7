# in-step A/B: ring attention output stores 16 B (product) vs 8 B (st8)
set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
VD=$GRAFT_REPO_ROOT/chunkformer_amd/_build/variants
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_parity.py 2>&1 | tail -1
for v in st8 prod st8 prod st8 prod; do
  if [ $v = prod ]; then unset CFM_LIB; else export CFM_LIB=$VD/libcfm_$v.so; fi
  timeout -k 10 300 python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/attst_b.json 2>/dev/null
  python3 -c "import json; d=json.loads(open('gpurun_out/attst_b.json').read().strip().splitlines()[-1]); b=d['breakdown_ms']; print('$v', d['value'], d['ms_per_step'], b['chunk_attention'])"
done
