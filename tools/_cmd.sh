set -e
mkdir -p gpurun_out
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread > gpurun_out/parity.log 2>&1
tail -2 gpurun_out/parity.log
for i in 1 2; do timeout -k 10 120 python3 tools/layer_bench.py --layers 1 --iters 3 | grep chunk_attention; done
