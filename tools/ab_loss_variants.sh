#!/usr/bin/env bash
# Alternated A/B of loss-head builds on one box: product, then each variant named in $VARIANTS
# (pipelinerl_amd/variants/libprl_hip_<name>.so), $ROUNDS times; lines in gpurun_out/ab_<name>_<i>.log
set -u
B="python bench.py --steps ${STEPS:-100} --warmup 10 --no-cpu-baseline --no-trainer-step --no-c3"
D=pipelinerl-swe_amd/pipelinerl_amd/variants
specs=()
for i in $(seq 1 ${ROUNDS:-3}); do
  specs+=("120:ab_product_$i:$B")
  for v in ${VARIANTS:-vec_row_inputs}; do specs+=("120:ab_${v}_$i:PRL_LIB=\$PWD/$D/libprl_hip_$v.so $B"); done
done
tools/gpu_steps.sh "${specs[@]}"
