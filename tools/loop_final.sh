# end-to-end loop on the final code with the reference config's gradient_checkpointing: true
# (auto policy): 1.5B at 16 k-token micro-batches and the C3 7B distribution -> gpurun_out/loop_session.jsonl
set -e
mkdir -p gpurun_out
timeout -k 10 400 python -u tools/loop_bench.py --model 1.5b --seq-length 16384 --samples-per-step 64 --steps 5 --grad-ckpt | grep '^{' >> gpurun_out/loop_session.jsonl
timeout -k 10 500 python -u tools/loop_bench.py --model 7b --dist c3 --seq-length 12000 --samples-per-step 16 --steps 4 --grad-ckpt | grep '^{' >> gpurun_out/loop_session.jsonl
