# fp32 loss head A/B: the part-resident kernel (product) vs the streaming kernel (PRL_HYB_NL=-1)
# (variant build: python -c "from pipelinerl_amd import _build; _build.build_variant('hyb_off', {'PRL_HYB_NL': '-1'})"),
# three alternating rounds, one line per run (tools/loss_dtype_bench.py)
set -u
V=pipelinerl-swe_amd/pipelinerl_amd/variants
for r in 1 2 3; do
  for arm in product off; do
    lib=""
    [ $arm = off ] && lib=$V/libprl_hip_hyb_off.so
    PRL_LIB=$lib timeout -k 10 120 python tools/loss_dtype_bench.py | grep float32 | sed "s/^{/{\"arm\": \"$arm\", \"round\": $r, /" || exit $?
  done
done
