# The fp32-master AdamW step's rocprofv3 evidence: kernel stats, then FETCH_SIZE / WRITE_SIZE in
# separate PMC passes (each under its own limit); CSVs under gpurun_out/prof_adamw, pmc_adamw_{fetch,write}.
set -u
export TMPDIR=/tmp
bash tools/prof_stats.sh prof_adamw 150 tools/adamw_master_bench.py --model 7b --steps 6 || exit $?
for c in FETCH_SIZE WRITE_SIZE; do
  d=pmc_adamw_$( [ $c = FETCH_SIZE ] && echo fetch || echo write )
  timeout -s KILL 150 rocprofv3 --pmc $c --output-format csv -d /tmp/$d -o run -- python3 tools/adamw_master_bench.py --model 7b --steps 2 > gpurun_out/$d.log 2>&1 || exit $?
  mkdir -p gpurun_out/$d
  find /tmp/$d -name "*counter_collection.csv" -exec cp {} gpurun_out/$d/ \;
done
