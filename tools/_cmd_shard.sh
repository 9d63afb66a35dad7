# §8(e) round check on one GPU: shard tests, the sharded bench at N=1 (configs[2], 980 min on one
# GPU) and a 2-rank rehearsal of the N>1 bench path on the one GPU over gloo (CFM_DIST_BACKEND).
set -e
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_sharded.py -x -v --timeout 200 --timeout-method thread > gpurun_out/gpu_shard.log 2>&1 || { tail -40 gpurun_out/gpu_shard.log; exit 1; }
tail -3 gpurun_out/gpu_shard.log
timeout -k 10 300 python3 bench.py --config sharded --no-cpu-baseline --steps 3 --warmup 1 > gpurun_out/bench_sharded1.log 2>&1 || { tail -20 gpurun_out/bench_sharded1.log; exit 1; }
tail -1 gpurun_out/bench_sharded1.log
CFM_DIST_BACKEND=gloo timeout -k 10 400 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 2 --warmup 1 --minutes 120 --no-breakdown > gpurun_out/bench_sharded2.log 2>&1 || { tail -30 gpurun_out/bench_sharded2.log; exit 1; }
tail -1 gpurun_out/bench_sharded2.log
