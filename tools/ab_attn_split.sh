# attention backward: heavy key blocks split over query heads (PRL_ATTN_SPLIT=1, default) vs one
# workgroup per key block (0), alternated on one box   -> gpurun_out/ab_attn_split.jsonl
set -e
mkdir -p gpurun_out
for s in 0 1 0 1; do
  PRL_ATTN_SPLIT=$s timeout -k 10 200 python -u tools/attn_bwd_bench.py lens 28 4 4096 8192 8192,8192 8511 3755,1617,6053 3160,3283 6122 4703,5963 6813,1243 4096,4096,2048,1760 2048,2048,2048,2048,2048,1760 \
    | sed "s/}$/, \"split\": $s}/" >> gpurun_out/ab_attn_split.jsonl
  PRL_ATTN_SPLIT=$s timeout -k 10 200 python -u tools/attn_bwd_bench.py lens 12 2 2048,2048,2048,2048,2048,2048,2048,2048 4096 8192,8192 \
    | sed "s/}$/, \"split\": $s}/" >> gpurun_out/ab_attn_split.jsonl
done
