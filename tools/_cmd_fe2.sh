# front-end: interleaved linear MFMAs; hi+lo vs hi-only
set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python3 -u -m pytest -x -q -s --timeout 300 --timeout-method thread tests/test_gpu_scale.py -k "golden_utterances or large_12L or window_groups" > gpurun_out/fe2.log 2>&1 || { tail -60 gpurun_out/fe2.log; exit 1; }
grep -E "golden utt|passed|failed" gpurun_out/fe2.log | tail -5
for v in "" linhi "" linhi; do
  if [ -n "$v" ]; then export CFM_LIB=$GRAFT_REPO_ROOT/chunkformer_amd/_build/variants/libcfm_$v.so; else unset CFM_LIB; fi
  timeout -k 10 300 python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/fe2_b.json 2>/dev/null
  python3 -c "import json; d=json.loads(open('gpurun_out/fe2_b.json').read().strip().splitlines()[-1]); b=d['breakdown_ms']; print('$v', d['value'], d['ms_per_step'], {k: b[k] for k in b if k.startswith('frontend')})"
done
