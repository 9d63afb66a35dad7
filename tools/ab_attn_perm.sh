# round 6: skew scratch rows in a permuted slot order (ATTN_SKEW_PERM) against query order, one process per arm
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_scale.py tests/test_gpu_model.py -m gpu -x -q --timeout 200 -k "ring_kernel_shapes or golden_utterances_inside or full_attention_mixed or golden" > gpurun_out/t_perm.log 2>&1 || { echo "tests FAILED"; tail -30 gpurun_out/t_perm.log; exit 1; }
echo "tests: $(tail -1 gpurun_out/t_perm.log)"
VARIANTS="${VARIANTS:-base noperm base2 nopermb}" BCFG=${BCFG:-full} bash tools/ab_prio.sh
