# whole-step A/B of this build against the round-5 build (.r5base/: its bench.py, python package and libcfm.so,
# built from commit a822257 by tools/ab_round.sh's caller), interleaved on one box
cd ${GRAFT_REPO_ROOT:-.}
for r in 1 2; do
  for v in r6 r5; do
    d=.; [ $v = r5 ] && d=.r5base
    (cd $d && timeout -k 10 300 python3 bench.py --no-cpu-baseline --steps 20 --warmup 5 ${BARGS:-} > $OLDPWD/gpurun_out/abr_${v}_$r.log 2>&1) || { echo "$v failed"; tail -5 gpurun_out/abr_${v}_$r.log; exit 1; }
    echo "$v run $r: $(grep '^{' gpurun_out/abr_${v}_$r.log | grep -o '"ms_per_step": [0-9.]*')"
  done
done
