cd $GRAFT_REPO_ROOT
for v in skrd52 rp56; do
  CFM_LIB=$PWD/chunkformer_amd/_build/variants/libcfm_$v.so timeout -k 10 300 python3 -u -m pytest tests/test_gpu_scale.py -m gpu -x -q --timeout 200 -k "ring_kernel_shapes or golden_utterances_inside or full_attention_mixed" > gpurun_out/t_$v.log 2>&1 || { echo "$v tests FAILED"; tail -20 gpurun_out/t_$v.log; exit 1; }
  echo "$v: $(tail -1 gpurun_out/t_$v.log)"
done
VARIANTS="base skrd52 rp56 base2 skrd52b" BCFG=full bash tools/ab_prio.sh
