set -e
for d in 0 1 3 4 6 7; do echo "== wst diag $d"; CFM_GEMM_DIAG=$d timeout -k 10 120 python3 tools/gemm_bench.py --iters 20 --only ffn_w1 2>&1 | grep -v amdgpu; done
echo "== 256 kernel"; CFM_GEMM_WST=0 timeout -k 10 120 python3 tools/gemm_bench.py --iters 20 2>&1 | grep -v amdgpu
echo "== wst"; timeout -k 10 120 python3 tools/gemm_bench.py --iters 20 2>&1 | grep -v amdgpu
