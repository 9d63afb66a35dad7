# Wave-state / instruction-mix PMC passes over ONE encoder layer (tools/layer_bench.py), summarised for
# the kernels whose names contain the given substrings.   bash tools/pmc_kernels.sh TAG substr...  (via gpurun)
set -e
T=${1:-kp}; shift
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/$T
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
LB="$R/tools/layer_bench.py --iters 1 ${LB_ARGS:-}"   # LB_ARGS: e.g. "--opt fe_conv=3"
timeout -k 10 200 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS --output-format csv -d $O/p1 -o p -- python3 $LB > $O/p1.log 2>&1
timeout -k 10 200 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_LDS_IDX_ACTIVE --output-format csv -d $O/p2 -o p -- python3 $LB > $O/p2.log 2>&1
timeout -k 10 200 rocprofv3 --pmc SQ_LDS_UNALIGNED_STALL SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_BUSY_CYCLES --output-format csv -d $O/p3 -o p -- python3 $LB > $O/p3.log 2>&1
python3 $R/tools/pmc_summary.py $O "$@" > $O/summary.txt 2>&1
cat $O/summary.txt
