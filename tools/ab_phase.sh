# Loss-head read/write phasing A/B (PRL_PHASED variants, tools/build_variants.py), alternated
# twice on one box   -> gpurun_out/ab_phase.jsonl
set -e
mkdir -p gpurun_out
V=pipelinerl-swe_amd/pipelinerl_amd/variants
B="python -u bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-trainer-step --no-c3"
for rep in 1 2; do
  for v in main unphased; do
    if [[ $v == main ]]; then unset PRL_LIB; else export PRL_LIB=$PWD/$V/libprl_hip_$v.so; fi
    timeout -k 10 120 $B | grep '^{' | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(json.dumps({'variant': '$v', 'value': d['value'], 'kernel_ms': d['roofline']['kernel_ms'], 'frac': d['roofline']['frac'], 'ms_per_step': d['ms_per_step']}))" >> gpurun_out/ab_phase.jsonl
  done
done
