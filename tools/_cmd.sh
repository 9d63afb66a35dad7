set -e
timeout -k 10 300 python -m pytest tests -m gpu -x -q > gpurun_out/gpu_tests6.log 2>&1
timeout -k 10 300 python3 tools/ab_bench.py --layers 2 --rounds 3 > gpurun_out/ab2.log 2>&1
