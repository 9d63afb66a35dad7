# Rehearsal of the N-rank bench on ONE GPU (both ranks share cuda:0, gloo collectives on host
# copies): exercises plan_shards, the per-rank encoder runs and the ids / log-prob gathers.
set -e
R=$GRAFT_REPO_ROOT
export CFM_DIST_BACKEND=gloo
timeout -k 10 400 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 $R/bench.py --gpus 2 --steps 2 --warmup 1 --minutes 120 --no-cpu-baseline > $R/gpurun_out/rehearse2.log 2>&1
tail -1 $R/gpurun_out/rehearse2.log | cut -c1-1200
