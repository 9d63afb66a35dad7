# FFN w2 (256x256 kernel) timing diagnostics: 1 no MFMA, 2 no DMA in the loop, 3 no epilogue
set -e
cd $GRAFT_REPO_ROOT
export CFM_LIB=$GRAFT_REPO_ROOT/chunkformer_amd/_build/variants/libcfm_diag.so
for dg in 0 1 2 3 0; do
  echo "== diag $dg"; timeout -k 10 120 python3 tools/gemm_bench.py --iters 20 --only ffn_w2 --diag $dg 2>&1 | grep -v amdgpu.ids
done
