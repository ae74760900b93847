#!/usr/bin/env bash
# Alternated A/B of the attention forward: product vs the variant named in $VARIANT (a
# pipelinerl_amd/variants/libprl_hip_<name>.so), attention GPU tests first, then
# tools/attn_bwd_bench.py three times per build and one C3 7B step each.
set -u
V=pipelinerl-swe_amd/pipelinerl_amd/variants/libprl_hip_${VARIANT:-head}.so
specs=("!400:attn_tests:python -u -m pytest tests/test_attn_bwd_gpu.py tests/test_model_ops_gpu.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider")
for i in 1 2 3; do
  specs+=("180:at_product_$i:python tools/attn_bwd_bench.py" "180:at_${VARIANT:-head}_$i:PRL_LIB=\$PWD/$V python tools/attn_bwd_bench.py")
done
specs+=("300:c3_product:python tools/c3_step.py --steps 3" "300:c3_${VARIANT:-head}:PRL_LIB=\$PWD/$V python tools/c3_step.py --steps 3")
tools/gpu_steps.sh "${specs[@]}"
