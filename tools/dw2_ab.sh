set -e
for v in base pipe0 unpk; do
  L=chunkformer_amd/_build/libcfm.so; case $v in base) ;; *) L=chunkformer_amd/_build/variants/libcfm_$v.so;; esac
  echo "== $v"; CFM_LIB=$PWD/$L timeout -k 10 300 python3 tools/dw2_probe.py 2>&1 | grep -v amdgpu.ids | grep fp16
done
