# A/B of the fused q/k/v projection (PRL_FUSED_QKV) on the C3 7B step and bench.py's 1.5B trainer
# step, interleaved, one box   -> gpurun_out/ab_fused_qkv.jsonl
set -e
mkdir -p gpurun_out
for v in 1 0 1 0; do
  PRL_FUSED_QKV=$v timeout -k 10 300 python -u tools/c3_step.py | grep '^{' | sed "s/}$/, \"fused_qkv\": $v, \"probe\": \"c3_dp\"}/" >> gpurun_out/ab_fused_qkv.jsonl
  PRL_FUSED_QKV=$v timeout -k 10 300 python -u bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-c3 | grep '^{' \
    | python -c "import sys,json; d=json.loads(sys.stdin.readline()); t=d['trainer_step']; t['fused_qkv']=$v; t['probe']='trainer_step'; print(json.dumps(t))" >> gpurun_out/ab_fused_qkv.jsonl
done
