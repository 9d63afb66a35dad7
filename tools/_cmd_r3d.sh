# round 3: head_dim 128 kernel checks: parity, A/B of score-loop variants, kernel stats of the 4-head bench
set -e
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd $R
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 200 --timeout-method thread "tests/test_gpu_scale.py::test_head_dim_128_kernel_vs_generic" "tests/test_gpu_scale.py::test_four_heads_head_dim_128" > gpurun_out/r3d_t.log 2>&1 || { tail -30 gpurun_out/r3d_t.log; exit 1; }
tail -1 gpurun_out/r3d_t.log
timeout -k 10 300 python3 tools/ab_bench.py --heads 4 --layers 12 --rounds 3 --variant attn128_var=0 --variant attn128_var=1 > gpurun_out/r3d_ab.log 2>&1
grep -E "variant|chunk_attention|total" gpurun_out/r3d_ab.log
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/r3d_prof -o b -- python3 $R/bench.py --heads 4 --steps 2 --warmup 1 --no-cpu-baseline --no-breakdown > $R/gpurun_out/r3d_prof.log 2>&1
f=$(find $R/gpurun_out/r3d_prof -name "*kernel_stats.csv" | head -1); head -12 $f | cut -c1-160
