# lm_head chunk size A/B on the 1.5B trainer micro-batch step (65 536 tokens, 57 344 label rows):
# 16 384-row chunks (fp32 dW accumulator) vs one chunk (bf16-output dW GEMM)
set -e
for c in 16384 65536 16384 65536; do
  timeout -k 10 200 python -u tools/trainer_step_bench.py --mode trainer --loss fused_head --tokens 65536 --steps 5 \
    --warmup 2 --chunk $c | sed "s/}$/, \"chunk\": $c}/" | grep '^{' >> gpurun_out/ab_chunk.jsonl
done
