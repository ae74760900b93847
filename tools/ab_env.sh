# Generic interleaved A/B of one environment switch on the C3 7B step (tools/c3_step.py) and
# bench.py's 1.5B trainer step, one box:
#   bash tools/ab_env.sh <VAR> [values...]   (default values: 0 1 0 1)  -> gpurun_out/ab_<var>.jsonl
# C3_ONLY=1 skips the trainer step.
set -e
var=$1; shift
vals=${*:-0 1 0 1}
out=gpurun_out/ab_$(echo "$var" | tr 'A-Z' 'a-z').jsonl
mkdir -p gpurun_out
for v in $vals; do
  env "$var=$v" timeout -k 10 300 python -u tools/c3_step.py --steps 4 | grep '^{' \
    | python -c "import sys,json; d=json.loads(sys.stdin.readline()); d['$var']='$v'; d['probe']='c3_dp'; print(json.dumps(d))" >> "$out"
  [ "${C3_ONLY:-0}" = 1 ] && continue
  env "$var=$v" timeout -k 10 300 python -u bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-c3 | grep '^{' \
    | python -c "import sys,json; d=json.loads(sys.stdin.readline()); t=d['trainer_step']; t['$var']='$v'; t['probe']='trainer_step'; print(json.dumps(t))" >> "$out"
done
