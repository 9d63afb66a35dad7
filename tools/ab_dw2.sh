# fused pw1 + dw2 front-end GEMM compile variants (DW2_RP_DEF ring pitch): bit-identity tests, then A/B
cd ${GRAFT_REPO_ROOT:-.}
for v in ${TESTV:-rp544 rp576}; do
  CFM_LIB=$PWD/chunkformer_amd/_build/variants/libcfm_$v.so timeout -k 10 300 python3 -u -m pytest tests/test_gpu_scale.py -m gpu -x -q --timeout 200 -k "frontend_fused or golden_utterances_inside" > gpurun_out/t_$v.log 2>&1 || { echo "$v tests FAILED"; tail -20 gpurun_out/t_$v.log; exit 1; }
  echo "$v: $(tail -1 gpurun_out/t_$v.log)"
done
VARIANTS="${VARIANTS:-base rp544 rp576 base2 rp544b}" CLASS=frontend_pw_gemm BCFG=${BCFG:-full} bash tools/ab_prio.sh
