# GEMM component timing on the encoder shapes: normal / no-MFMA / no-DMA-wait / no-epilogue /
# no-store builds (cfm_op_gemm variant bits 8-15) + hipBLASLt reference.  Run via gpurun from the
# repo root:  bash tools/gemm_diag.sh [only-shape]
set -e
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/gemm_diag
mkdir -p $O
ONLY=${1:+--only $1}
for d in 0 1 2 3 5; do
  timeout -k 10 120 python3 $R/tools/gemm_bench.py --iters 20 --diag $d $ONLY > $O/diag$d.log 2>&1
done
timeout -k 10 120 python3 $R/tools/torch_gemm_ref.py > $O/hipblaslt.log 2>&1
