# PMC passes over ONE encoder layer of the bench workload (tools/layer_bench.py): clock, wave-state
# split, MFMA/LDS, L2 hit/miss, HBM fetch/write.  bash tools/layer_pmc.sh TAG   (via gpurun)
set -e
T=${1:-lp}
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/$T
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
LB="$R/tools/layer_bench.py --iters 1"
timeout -k 10 200 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY --output-format csv -d $O/p1 -o p -- python3 $LB > $O/p1.log 2>&1
timeout -k 10 200 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS --output-format csv -d $O/p2 -o p -- python3 $LB > $O/p2.log 2>&1
timeout -k 10 200 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum --output-format csv -d $O/p3 -o p -- python3 $LB > $O/p3.log 2>&1
timeout -k 10 200 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/p4 -o p -- python3 $LB > $O/p4.log 2>&1
timeout -k 10 200 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/p5 -o p -- python3 $LB > $O/p5.log 2>&1
python3 $R/tools/pmc_summary.py $O ffn_fused chunk_attention > $O/summary.txt 2>&1 || true
