# GEMM paths at endless_decode's tbd-1800 segment size (12,736 rows): default / 128-tile / no weight-stationary
set -e
R=$GRAFT_REPO_ROOT
cd $R
for v in "" "--small" "--wst 7" "--wst 2"; do
  echo "== $v"
  timeout -k 10 120 python3 tools/gemm_bench.py --m 12736 --iters 20 --only ffn_w1,ffn_w2,qkv,out/pw2,pw1_glu $v 2>&1 | grep -v amdgpu.ids
done
