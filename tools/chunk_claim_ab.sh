# The 1.5B micro-batch trainer step (C2's 65 536 tokens, fused label-row loss head) with the phased
# SwiGLU kernels claiming chunks (default) and with the static stride (PRL_CHUNK_CLAIM=0), three
# alternated rounds: bash tools/chunk_claim_ab.sh  -> gpurun_out/chunk_claim_ab.jsonl
set -u
B="python tools/trainer_step_bench.py --mode trainer --model 1.5b --tokens 65536 --loss fused_head --steps 4 --warmup 1"
for r in 1 2 3; do
  for arm in claim static; do
    if [ $arm = static ]; then pre="PRL_CHUNK_CLAIM=0"; else pre=""; fi
    line=$(env $pre timeout -k 10 240 $B 2>/dev/null | grep '^{') || exit $?
    echo "{\"round\": $r, \"arm\": \"$arm\", \"line\": $line}" >> gpurun_out/chunk_claim_ab.jsonl
  done
done
