# dense attention 16-B stores: parity + configs[4] A/B
set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
VD=$GRAFT_REPO_ROOT/chunkformer_amd/_build/variants
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_scale.py -k "dense or full or ring" 2>&1 | tail -1
for v in st8 prod st8 prod; do
  if [ $v = prod ]; then unset CFM_LIB; else export CFM_LIB=$VD/libcfm_$v.so; fi
  timeout -k 10 300 python3 bench.py --config full --steps 5 --warmup 2 > gpurun_out/attst2_b.json 2>/dev/null
  python3 -c "import json; d=json.loads(open('gpurun_out/attst2_b.json').read().strip().splitlines()[-1]); print('$v', d['value'], d['ms_per_step'], d['roofline']['avg_launch_ms'])"
done
