set -e
timeout -k 10 300 python -m pytest tests -m gpu -x -q > gpurun_out/gpu_tests3.log 2>&1
for a in 0 1 2 3; do timeout -k 10 120 python3 tools/layer_bench.py --iters 2 --opt attn_diag=$a > gpurun_out/attn3_d$a.log 2>&1; done
