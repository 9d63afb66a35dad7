set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 400 python3 -u tools/split_bench.py --parts 2 --parts 3 --parts 4 --rounds 4 2>&1 | grep -v amdgpu.ids | tee gpurun_out/split.log
