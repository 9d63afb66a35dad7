# ring-attention variant A/B: parity tests on the variant library, then one process per arm (tools/ab_prio.sh)
# usage: VAR=ovl2 bash tools/ab_attn_var.sh
cd $GRAFT_REPO_ROOT
CFM_LIB=$PWD/chunkformer_amd/_build/variants/libcfm_$VAR.so timeout -k 10 300 python3 -u -m pytest tests/test_gpu_scale.py tests/test_gpu_model.py -m gpu -x -q --timeout 200 -k "ring_kernel_shapes or golden_utterances_inside or full_attention_mixed or golden" > gpurun_out/t_$VAR.log 2>&1 || { echo "$VAR tests FAILED"; tail -30 gpurun_out/t_$VAR.log; exit 1; }
echo "$VAR tests: $(tail -1 gpurun_out/t_$VAR.log)"
VARIANTS="base $VAR base2 ${VAR}b" BCFG=${BCFG:-masked} bash tools/ab_prio.sh
