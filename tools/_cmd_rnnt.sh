# RNN-T consumer timing (small cases; B = 1 is the sequential worst case)
set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for fb in "500 1" "2000 1" "500 64" "500 256"; do
  set -- $fb
  timeout -k 10 120 python3 -u tools/rnnt_bench.py --frames $1 --batch $2 2>&1 | grep -v amdgpu.ids | tee -a gpurun_out/rnnt.txt
done
