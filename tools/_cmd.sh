set -e
timeout -k 10 300 python3 tools/ab_bench.py --layers 2 --rounds 3 --variant fused_ffn=1,ffn_variant=0 --variant fused_ffn=1,ffn_variant=1 --variant fused_ffn=0 > gpurun_out/ab1.log 2>&1
