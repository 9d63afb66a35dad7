# Run several pytest selections of the GPU suite, each in its own process, one after another; a crash in one
# (exit status recorded) does not stop the others.   bash tools/pytest_probe.sh "expr1" "expr2" ...  (via gpurun)
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
O=$R/gpurun_out/probe
mkdir -p $O
cd $R
i=0
for e in "$@"; do
  i=$((i + 1))
  timeout -k 10 300 python3 -u -m pytest tests -m gpu -x -q ${PROBE_ARGS:---timeout 240 --timeout-method thread} -k "$e" > $O/p$i.log 2>&1
  rc=$?
  echo "[$e] rc=$rc $(grep -E 'passed|failed' $O/p$i.log | tail -1) $(grep -m1 -E 'Fatal Python error' $O/p$i.log)"
  grep -B2 -m1 "Fatal Python error" $O/p$i.log | head -3
  [ $rc -eq 124 ] && break
done
exit 0
