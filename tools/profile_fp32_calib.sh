# FETCH_SIZE / WRITE_SIZE calibration of the fp32 loss head (tools/fetch_calibration.py): one pass
# per counter, each under its own limit; the counter CSVs under gpurun_out/calib_{fetch,write}/.
set -u
export TMPDIR=/tmp
for c in FETCH_SIZE WRITE_SIZE; do
  d=calib_$( [ $c = FETCH_SIZE ] && echo fetch || echo write )
  timeout -s KILL 240 rocprofv3 --pmc $c --output-format csv -d /tmp/$d -o run -- python3 tools/fetch_calibration.py --reps 3 > gpurun_out/$d.log 2>&1 || exit $?
  mkdir -p gpurun_out/$d
  find /tmp/$d -name "*counter_collection.csv" -exec cp {} gpurun_out/$d/ \;
done
