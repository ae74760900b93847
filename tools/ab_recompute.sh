# gradient_checkpointing: true (the reference config) with the recompute policy "always" (the
# reference's behaviour) vs "auto" (skip it when the activations fit; finetune/recompute.py), on the
# end-to-end loop, alternated on one box   -> gpurun_out/ab_recompute.jsonl
set -e
mkdir -p gpurun_out
for p in always auto always auto; do
  timeout -k 10 500 python -u tools/loop_bench.py --model 7b --dist c3 --seq-length 12000 --samples-per-step 16 --steps 4 \
    --grad-ckpt --ckpt-policy $p | grep '^{' >> gpurun_out/ab_recompute.jsonl
done
for p in always auto; do
  timeout -k 10 400 python -u tools/loop_bench.py --model 1.5b --seq-length 16384 --samples-per-step 64 --steps 4 \
    --grad-ckpt --ckpt-policy $p | grep '^{' >> gpurun_out/ab_recompute.jsonl
done
