# PMC passes on the GEMM micro-benchmark (one shape): clock, wave-state split, MFMA busy, LDS.
#   bash tools/gemm_pmc.sh ffn_w1   (via gpurun, from the repo root)
set -e
S=${1:-ffn_w1}
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/gemm_pmc_$S
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
GB="$R/tools/gemm_bench.py --iters 3 --only $S"
timeout -k 10 200 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY --output-format csv -d $O/p1 -o p -- python3 $GB > $O/p1.log 2>&1
timeout -k 10 200 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS --output-format csv -d $O/p2 -o p -- python3 $GB > $O/p2.log 2>&1
timeout -k 10 200 rocprofv3 --pmc SQ_LDS_IDX_ACTIVE SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SALU --output-format csv -d $O/p3 -o p -- python3 $GB > $O/p3.log 2>&1
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt -o k -- python3 $GB > $O/kt.log 2>&1
python3 $R/tools/pmc_summary.py $O > $O/summary.txt 2>&1 || true
