set -e
mkdir -p gpurun_out
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_model.py -x -v --timeout 120 --timeout-method thread > gpurun_out/gpu_tests_model.log 2>&1
timeout -k 10 300 python3 bench.py --config endless --steps 2 --warmup 1 > gpurun_out/bench_endless.log 2>&1
timeout -k 10 300 python3 bench.py --config full --steps 3 --warmup 1 > gpurun_out/bench_full.log 2>&1
tail -1 gpurun_out/bench_endless.log
tail -1 gpurun_out/bench_full.log
