#!/usr/bin/env bash
# A/B the experiment builds in pipelinerl_amd/variants/ with bench.py (one process each).
set -u
for so in pipelinerl-swe_amd/pipelinerl_amd/variants/libprl_hip_*.so; do
  name=$(basename "$so" .so); name=${name#libprl_hip_}
  echo "=== variant $name"
  PRL_LIB="$PWD/$so" timeout -k 10 240 python bench.py --steps 20 --warmup 3 --no-cpu-baseline > "gpurun_out/variant_$name.json" 2> "gpurun_out/variant_$name.err"
  rc=$?
  echo "rc=$rc"; tail -c 600 "gpurun_out/variant_$name.json"; echo
  case $rc in 0) ;; *) echo "stopping after rc=$rc"; exit $rc ;; esac
done
