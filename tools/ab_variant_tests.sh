# Correctness of A/B library variants (a pytest -k expression under each CFM_LIB variant, stops at the first
# failure), then the tools/ab_prio.sh timing.   VARIANTS="v1 v2" KEXPR="ring" CLASS=... bash tools/ab_variant_tests.sh
set -e
O=gpurun_out; mkdir -p $O
for v in $VARIANTS; do
  CFM_LIB=$PWD/chunkformer_amd/_build/variants/libcfm_$v.so timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q \
    --timeout 300 --timeout-method thread -k "$KEXPR" > $O/abt_$v.log 2>&1 || { echo "$v FAILED"; tail -20 $O/abt_$v.log; exit 1; }
  echo "$v: $(tail -1 $O/abt_$v.log)"
done
VARIANTS="base $VARIANTS base2 ${VARIANTS}2" bash tools/ab_prio.sh
