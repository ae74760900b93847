# The trainer-side half of "weight broadcast fully overlapped", profiled: the C3 7B step with the
# weight-update snapshot in flight (tools/c3_step.py --snapshot) under rocprofv3 --kernel-trace, then
# how much of each snapshot (prl_flatten_bf16 call) ran beside the step's own kernels
# (tools/kernel_overlap.py; the first 4 calls are the snapshot-alone timing and are left out).
# Outputs under gpurun_out/snap: the probe's JSON line, kernel stats, the overlap summary.
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out/snap
timeout -k 10 ${1:-600} rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/prof_snap -o run -- \
  python3 tools/c3_step.py --snapshot > gpurun_out/snap/c3_step.log 2>&1 || exit $?
grep '^{' gpurun_out/snap/c3_step.log > gpurun_out/snap/c3_step.jsonl
find /tmp/prof_snap -name "*_stats.csv" -exec cp {} gpurun_out/snap/ \;
trace=$(find /tmp/prof_snap -name "*kernel_trace.csv" -print -quit)
python3 tools/kernel_overlap.py "$trace" flatten_bf16 --skip-first-calls 4 --out gpurun_out/snap/overlap.json
