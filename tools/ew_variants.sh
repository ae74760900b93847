# element-wise kernel A/B over the experiment builds: the in-tree library, then each variant .so
#   bash tools/ew_variants.sh [ew_bench args]   -> gpurun_out/ew_variants.jsonl
set -u
mkdir -p gpurun_out
for rep in 1 2; do
for so in "" pipelinerl-swe_amd/pipelinerl_amd/variants/libprl_hip_*.so; do
  name=main; [ -n "$so" ] && { name=$(basename "$so" .so); name=${name#libprl_hip_}; }
  PRL_LIB=${so:+$PWD/$so} timeout -k 10 120 python tools/ew_bench.py "$@" > gpurun_out/ew_v.tmp 2>> gpurun_out/ew_variants.err
  rc=$?
  sed "s/}$/, \"variant\": \"$name\"}/" gpurun_out/ew_v.tmp | grep '^{' >> gpurun_out/ew_variants.jsonl
  case $rc in 0) ;; *) echo "stopping after rc=$rc ($name)"; exit $rc ;; esac
done
done
