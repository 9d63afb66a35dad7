# PMC of the front-end kernels over one layer of the bench workload
set -e
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/fepmc
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
LB="$R/tools/layer_bench.py --iters 1"
timeout -s KILL 200 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAVES --output-format csv -d $O/p1 -o p -- python3 $LB > $O/p1.log 2>&1
timeout -s KILL 200 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_INST_CYCLES_VMEM --output-format csv -d $O/p2 -o p -- python3 $LB > $O/p2.log 2>&1
timeout -s KILL 200 rocprofv3 --pmc SQ_ACTIVE_INST_MISC SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_INSTS_SALU SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD SQ_ACTIVE_INST_EXP SQ_ACTIVE_INST_FLAT --output-format csv -d $O/p3 -o p -- python3 $LB > $O/p3.log 2>&1
python3 $R/tools/pmc_summary.py $O fe_conv0 fe_dw2 "gemm_wsp_kernel<0, 1" > $O/summary.txt 2>&1
cat $O/summary.txt
