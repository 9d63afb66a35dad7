set -e
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_ctc.py tests/test_gpu_model.py tests/test_gpu_checkpoint.py -x -v --timeout 120 --timeout-method thread > gpurun_out/gpu_ctc.log 2>&1 || { tail -40 gpurun_out/gpu_ctc.log; exit 1; }
tail -3 gpurun_out/gpu_ctc.log
timeout -k 10 300 python3 bench.py --no-cpu-baseline > gpurun_out/bench.log 2>&1 || { tail -20 gpurun_out/bench.log; exit 1; }
tail -1 gpurun_out/bench.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], d['ctc_ms'], d['roofline']['frac'])"
