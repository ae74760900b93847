# End-to-end loop throughput on the current code: 1.5B (16 k-token micro-batches) and the C3 7B
# distribution (12 000-token packing cap)   -> gpurun_out/loop_session.jsonl
set -e
mkdir -p gpurun_out
timeout -k 10 400 python -u tools/loop_bench.py --model 1.5b --seq-length 16384 --samples-per-step 64 --steps 5 | grep '^{' >> gpurun_out/loop_session.jsonl
timeout -k 10 500 python -u tools/loop_bench.py --model 7b --dist c3 --seq-length 12000 --samples-per-step 16 --steps 4 | grep '^{' >> gpurun_out/loop_session.jsonl
