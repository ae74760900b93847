# Two rocprofv3 --pmc passes (8 SQ counters each at most, never combined with tracing) over the
# packed attention at the 7B's heads (28 / 4) on two 8192-token sequences; counter CSVs under
# gpurun_out/attn_pmc{1,2}/.  Then: python tools/attn_pmc.py gpurun_out/attn_pmc1 gpurun_out/attn_pmc2
set -u
export TMPDIR=/tmp
P1="SQ_WAVE_CYCLES SQ_BUSY_CU_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_LDS"
P2="SQ_WAVE_CYCLES SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_MISC"
n=1
for P in "$P1" "$P2"; do
  timeout -s KILL 120 rocprofv3 --pmc $P --output-format csv -d /tmp/attn_pmc$n -o run -- python3 tools/attn_bwd_bench.py 16384 8192 28 4 > gpurun_out/attn_pmc$n.log 2>&1 || exit $?
  mkdir -p gpurun_out/attn_pmc$n
  find /tmp/attn_pmc$n -name "*counter_collection.csv" -exec cp {} gpurun_out/attn_pmc$n/ \;
  n=$((n + 1))
done
