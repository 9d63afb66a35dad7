set -e
O=gpurun_out; mkdir -p $O
for v in ${VARIANTS:-base prio1 prio2 base2}; do
  L=chunkformer_amd/_build/libcfm.so; case $v in base*) ;; *) L=chunkformer_amd/_build/variants/libcfm_${v%b}.so;; esac
  CFM_LIB=$PWD/$L timeout -k 10 300 python3 tools/ab_bench.py --layers 12 --rounds 3 > $O/abp_$v.log 2>&1
  grep -E "total|${CLASS:-chunk_attention}" $O/abp_$v.log | sed "s/^/$v /"
  CFM_LIB=$PWD/$L timeout -k 10 300 python3 bench.py --config ${BCFG:-full} --no-cpu-baseline --no-breakdown --steps 10 > $O/abf_$v.log 2>&1
  grep '^{' $O/abf_$v.log | grep -o '"value": [0-9.]*' | sed "s/^/$v full /"
done
