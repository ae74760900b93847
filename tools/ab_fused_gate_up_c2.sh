# A/B of the fused gate/up projection on bench.py's trainer_step (1.5B, 2 x 65 536-token micro-batches)
#   -> gpurun_out/ab_fused_gate_up_c2.jsonl
set -e
mkdir -p gpurun_out
for v in 1 0 1 0; do
  PRL_FUSED_GATE_UP=$v timeout -k 10 300 python -u bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-c3 | grep '^{' \
    | python -c "import sys,json; d=json.loads(sys.stdin.readline()); t=d['trainer_step']; t['fused_gate_up']=$v; print(json.dumps(t))" >> gpurun_out/ab_fused_gate_up_c2.jsonl
done
