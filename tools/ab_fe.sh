# front-end conv0+dw1 compile variants: the 240-min golden / kernel-agreement tests on the variant, then
# one-process A/B timings (tools/ab_prio.sh)
cd ${GRAFT_REPO_ROOT:-.}
for v in ${TESTV:-fed}; do
  CFM_LIB=$PWD/chunkformer_amd/_build/variants/libcfm_$v.so timeout -k 10 300 python3 -u -m pytest tests/test_gpu_scale.py -m gpu -x -q --timeout 200 -k "frontend or golden_utterances_inside" > gpurun_out/t_$v.log 2>&1 || { echo "$v tests FAILED"; tail -20 gpurun_out/t_$v.log; exit 1; }
  echo "$v: $(tail -1 gpurun_out/t_$v.log)"
done
VARIANTS="${VARIANTS:-base fed base2 fedb}" CLASS=frontend_conv0_dw BCFG=${BCFG:-full} bash tools/ab_prio.sh
