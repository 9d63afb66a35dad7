set -e
timeout -k 10 300 python -m pytest tests/test_gpu_ops.py -x -q -k ffn > gpurun_out/ffn_test.log 2>&1
timeout -k 10 300 python -m pytest tests -m gpu -x -q > gpurun_out/gpu_tests4.log 2>&1
timeout -k 10 300 python3 bench.py --no-cpu-baseline > gpurun_out/bench4.log 2>&1
