# fp32 loss head A/B: the part-resident kernel (product) vs the streaming kernel (PRL_HYB_NL=-1)
# vs the next-row prefetch (PRL_HYB_PREFETCH=1), three alternating rounds, one line per run (tools/loss_dtype_bench.py)
set -u
V=pipelinerl-swe_amd/pipelinerl_amd/variants
for r in 1 2 3; do
  for arm in product off pf1; do
    lib=""
    [ $arm = off ] && lib=$V/libprl_hip_hyb_off.so
    [ $arm = pf1 ] && lib=$V/libprl_hip_hyb_pf1.so
    PRL_LIB=$lib timeout -k 10 120 python tools/loss_dtype_bench.py | grep float32 | sed "s/^{/{\"arm\": \"$arm\", \"round\": $r, /" || exit $?
  done
done
