# Rehearsal of the N-rank bench on ONE GPU (both ranks share cuda:0, gloo collectives on host
# copies): a plain `bench.py --gpus 2` starts torch.distributed.run itself (bench.spawn_ranks),
# which exercises plan_shards, the per-rank encoder runs, the ids / log-prob gathers and the
# end-to-end timing.  The numbers are NOT a scaling measurement (two ranks share one GPU).
set -e
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
export CFM_DIST_BACKEND=gloo
timeout -k 10 400 python3 $R/bench.py --gpus 2 --steps 2 --warmup 1 --no-cpu-baseline > $R/gpurun_out/rehearse2.log 2>&1
grep '^{' $R/gpurun_out/rehearse2.log | tail -1 | cut -c1-1500
