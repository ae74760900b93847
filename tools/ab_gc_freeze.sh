# A/B of freezing the set-up heap before the first step (pipelinerl_amd/hostgc.py, PRL_GC_FREEZE)
# on the C3 7B step (with the host's garbage collections inside the timed steps counted) and,
# unless C3_ONLY=1, bench.py's 1.5B trainer step, interleaved, one box -> gpurun_out/ab_gc_freeze.jsonl
set -e
mkdir -p gpurun_out
for v in 0 1 0 1; do
  PRL_GC_FREEZE=$v timeout -k 10 300 python -u tools/c3_step.py --steps 4 | grep '^{' | sed "s/}$/, \"gc_freeze\": $v, \"probe\": \"c3_dp\"}/" >> gpurun_out/ab_gc_freeze.jsonl
  [ "${C3_ONLY:-0}" = 1 ] && continue
  PRL_GC_FREEZE=$v timeout -k 10 300 python -u bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-c3 | grep '^{' \
    | python -c "import sys,json; d=json.loads(sys.stdin.readline()); t=d['trainer_step']; t['gc_freeze']=$v; t['probe']='trainer_step'; print(json.dumps(t))" >> gpurun_out/ab_gc_freeze.jsonl
done
