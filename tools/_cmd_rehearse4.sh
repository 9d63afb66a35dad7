# Rehearsal of the 4-rank bench on ONE GPU (gloo collectives; not a scaling measurement)
set -e
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
export CFM_DIST_BACKEND=gloo
timeout -k 10 500 python3 -u $R/bench.py --gpus 4 --steps 2 --warmup 1 --no-cpu-baseline > $R/gpurun_out/rehearse4.log 2>&1
grep '^{' $R/gpurun_out/rehearse4.log | tail -1 | python3 -c "import sys,json; d=json.loads(sys.stdin.read()); print(d['n_gpus'], d['value'], d['ms_per_step'], d['end_to_end_ms'], d['allgather_ids_ms'], d['config']['chunks_rank0'])"
