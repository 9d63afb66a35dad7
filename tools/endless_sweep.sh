# configs[3] tbd 1800 pipeline-option sweep (one bench line per setting, one process each)
cd $GRAFT_REPO_ROOT
O=gpurun_out; mkdir -p $O
for a in "--pipeline-depth 4" "--pipeline-depth 3" "--pipeline-depth 5" "--pipe-opt attn_min_chunks=8" "--pipe-opt attn_min_chunks=32" "--pipe-opt wsp_small_div=2" "--pipeline-depth 4"; do
  timeout -k 10 300 python3 bench.py --config endless --tbd 1800 --no-cpu-baseline --no-breakdown $a > $O/es.log 2>&1 || { tail -5 $O/es.log; exit 1; }
  echo "$a: $(grep '^{' $O/es.log | grep -o '"value": [0-9.]*')"
done
