# round-3 profile refresh + RNN-T consumer timing
set -e
cd $GRAFT_REPO_ROOT
bash tools/_cmd_r3prof.sh
timeout -k 10 120 python3 -u tools/rnnt_bench.py --frames 500 --batch 1 2>&1 | grep -v amdgpu.ids | tee gpurun_out/prof_r03/rnnt.txt
timeout -k 10 120 python3 -u tools/rnnt_bench.py --frames 500 --batch 128 2>&1 | grep -v amdgpu.ids | tee -a gpurun_out/prof_r03/rnnt.txt
