# PMC passes (wave states, LDS instructions / bank conflicts, VALU) over one encoder layer of the bench
# workload (tools/layer_bench.py), for the front-end kernels.  bash tools/fe_prof.sh  (via gpurun)
set -e
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
LB="$R/tools/layer_bench.py --iters 1"
timeout -k 10 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VALU --output-format csv -d $R/gpurun_out/pmc_sq -o sq -- python $LB > /dev/null 2>&1
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $R/gpurun_out/pmc_w -o w -- python $LB > /dev/null 2>&1
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $R/gpurun_out/pmc_f -o f -- python $LB > /dev/null 2>&1
timeout -k 10 300 rocprofv3 --pmc SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SALU SQ_INSTS_SMEM SQ_WAIT_INST_LDS SQ_INSTS_MFMA --output-format csv -d $R/gpurun_out/pmc_sq2 -o sq2 -- python $LB > /dev/null 2>&1
