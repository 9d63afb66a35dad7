# A/B: weight-stationary GEMM with one barrier per two K-steps
set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
V=$GRAFT_REPO_ROOT/chunkformer_amd/_build/variants/libcfm_bar2.so
for r in 1 2; do
  echo "== base"; timeout -k 10 120 python3 tools/gemm_bench.py --iters 20 --only ffn_w1,qkv,out/pw2,pw1_glu,fe_pw1 2>&1 | grep -v amdgpu.ids
  echo "== bar2"; CFM_LIB=$V timeout -k 10 120 python3 tools/gemm_bench.py --iters 20 --only ffn_w1,qkv,out/pw2,pw1_glu,fe_pw1 2>&1 | grep -v amdgpu.ids
done
CFM_LIB=$V timeout -k 10 300 python3 -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_ops.py 2>&1 | tail -2
