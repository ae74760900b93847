# The bench's rocprofv3 evidence: kernel stats of the loss-head bench, then FETCH_SIZE and
# WRITE_SIZE in separate PMC passes (never combined with tracing; each pass under its own limit).
# Outputs (small CSVs only) under gpurun_out/prof_bench, gpurun_out/pmc_fetch, gpurun_out/pmc_write.
# The bench's N = 1 loss_head_fp32 probe runs in every pass: the fp32 kernels (pair + hybrid A/B) are
# profiled and counted beside the bf16 one.
set -u
export TMPDIR=/tmp
B="bench.py --steps 47 --warmup 3 --no-cpu-baseline --no-trainer-step --no-c3"
bash tools/prof_stats.sh prof_bench 240 $B || exit $?
for c in FETCH_SIZE WRITE_SIZE; do
  d=pmc_$( [ $c = FETCH_SIZE ] && echo fetch || echo write )
  timeout -s KILL 150 rocprofv3 --pmc $c --output-format csv -d /tmp/$d -o run -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-trainer-step --no-c3 > gpurun_out/$d.log 2>&1 || exit $?
  mkdir -p gpurun_out/$d
  find /tmp/$d -name "*counter_collection.csv" -exec cp {} gpurun_out/$d/ \;
done
