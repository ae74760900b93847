# C3 7B trainer step with the attention backward's heavy key blocks split (PRL_ATTN_SPLIT=1) vs not,
# alternated on one box   -> gpurun_out/ab_c3_split.jsonl
set -e
mkdir -p gpurun_out
for s in 0 1 0 1; do
  PRL_ATTN_SPLIT=$s timeout -k 10 300 python -u tools/c3_step.py | grep '^{' | sed "s/}$/, \"attn_split\": $s}/" >> gpurun_out/ab_c3_split.jsonl
done
