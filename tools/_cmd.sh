set -e
timeout -k 10 300 python3 tools/ab_bench.py --layers 2 --rounds 3 --variant gemm_variant=0 --variant gemm_variant=5 --variant gemm_variant=6 > gpurun_out/ab3.log 2>&1
