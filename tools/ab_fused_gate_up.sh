# A/B of the fused gate/up projection (PRL_FUSED_GATE_UP) on the C3 7B step, interleaved, one box
#   -> gpurun_out/ab_fused_gate_up.jsonl
set -e
mkdir -p gpurun_out
for v in 1 0 1 0; do
  PRL_FUSED_GATE_UP=$v timeout -k 10 300 python -u tools/c3_step.py | grep '^{' | sed "s/}$/, \"fused_gate_up\": $v}/" >> gpurun_out/ab_fused_gate_up.jsonl
done
