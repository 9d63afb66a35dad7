# A/B of ring-attention compile variants (tools/build_variant.py TAG attention.hip -D...): ab_bench over 12
# layers of the 240-min batch, per variant one process, base twice
cd ${GRAFT_REPO_ROOT:-.}
VARIANTS="${VARIANTS:-base prio0 prio2 kpf0 st8 base2}" BCFG=${BCFG:-full} bash tools/ab_prio.sh
