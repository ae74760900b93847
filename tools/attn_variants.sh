# attention backward A/B over the experiment builds: the in-tree library, then each variant .so
#   bash tools/attn_variants.sh "<T seq H Hkv>" ...   -> gpurun_out/attn_variants.jsonl
set -u
mkdir -p gpurun_out
for cfg in "$@"; do
  for so in "" pipelinerl-swe_amd/pipelinerl_amd/variants/libprl_hip_*.so; do
    name=main; [ -n "$so" ] && { name=$(basename "$so" .so); name=${name#libprl_hip_}; }
    PRL_LIB=${so:+$PWD/$so} timeout -k 10 120 python tools/attn_bwd_bench.py $cfg > gpurun_out/attn_v.tmp 2>> gpurun_out/attn_variants.err
    rc=$?
    sed "s/}$/, \"variant\": \"$name\"}/" gpurun_out/attn_v.tmp | grep '^{' >> gpurun_out/attn_variants.jsonl
    case $rc in 0) ;; *) echo "stopping after rc=$rc ($name $cfg)"; exit $rc ;; esac
  done
done
