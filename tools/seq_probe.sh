# tools/endless_seq.py under several step lists, each in its own process (via gpurun)
cd ${GRAFT_REPO_ROOT:-.}
for s in "$@"; do
  timeout -k 10 200 python3 tools/endless_seq.py "$s" > gpurun_out/seq.log 2>&1
  echo "[$s] rc=$? $(grep -c '^ok' gpurun_out/seq.log) ok; $(grep -m1 'Fatal' gpurun_out/seq.log)"
  grep "^call" gpurun_out/seq.log | tail -2
done
exit 0
