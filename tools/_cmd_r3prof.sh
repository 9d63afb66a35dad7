# round 3 profile set: rocprof kernel stats + PMC traffic + MFMA busy of the headline bench,
# then one bench line per config (masked, 4-head, endless tbd 1800 and 7200, full, fbank)
set -e
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/prof_r03
mkdir -p $O
bash $R/tools/profile_round.sh r03
cd $R
timeout -k 10 300 python3 bench.py --heads 4 --steps 10 --warmup 3 --no-cpu-baseline > $O/bench_4h.log 2>&1
timeout -k 10 400 python3 bench.py --config endless --tbd 1800 --steps 2 --warmup 1 > $O/bench_endless1800.log 2>&1
timeout -k 10 400 python3 bench.py --config endless --tbd 7200 --steps 2 --warmup 1 > $O/bench_endless7200.log 2>&1
timeout -k 10 300 python3 bench.py --config full --steps 5 --warmup 2 > $O/bench_full.log 2>&1
for f in bench bench_4h bench_endless1800 bench_endless7200 bench_full; do grep '^{' $O/$f.log | tail -1 | cut -c1-200; done
