# in-step A/B of the per-model kernel options (real activations; random-data microbenchmarks
# mislead at power-limited clocks)
set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
run() {
  timeout -k 10 300 python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline "$@" > gpurun_out/knob_b.json 2>/dev/null
  python3 -c "import json,sys; d=json.loads(open('gpurun_out/knob_b.json').read().strip().splitlines()[-1]); print(sys.argv[1:], d['value'], d['ms_per_step'], d['roofline']['frac'])" "$@"
}
run
run --opt col_group=1
run --opt col_group=2
run --opt nt_sites=0
run --opt nt_sites=14
run --opt nt_sites=24
run --opt nt_sites=72
run --opt store_mode=1
run --opt attn_reuse=0
run --opt conv_dma=0
run
