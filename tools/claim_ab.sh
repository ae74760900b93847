# The bf16 loss head with rows claimed from a counter (default) and with the static row stride
# (PRL_ROW_CLAIM=0), the bench's C2 line alternated three rounds: bash tools/claim_ab.sh
#   -> gpurun_out/claim_ab.jsonl
set -u
B="python bench.py --steps 30 --warmup 5 --no-cpu-baseline --no-trainer-step --no-c3 --no-fp32"
for r in 1 2 3; do
  for arm in claim static; do
    if [ $arm = static ]; then pre="PRL_ROW_CLAIM=0"; else pre=""; fi
    line=$(env $pre timeout -k 10 120 $B 2>/dev/null | grep '^{') || exit $?
    echo "{\"round\": $r, \"arm\": \"$arm\", \"line\": $line}" >> gpurun_out/claim_ab.jsonl
  done
done
