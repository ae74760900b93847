# Loop A/B of the loader's decode: libprl_data (native, GIL released, pinned) vs json + the
# PipelineBatchEncoding validators (PRL_NATIVE_DECODE=0), interleaved, one box.
#   bash tools/ab_decode.sh [seq_length] [steps]   -> gpurun_out/ab_decode.jsonl
set -e
S=${1:-16384}; N=${2:-5}
mkdir -p gpurun_out
for v in 1 0 1 0; do
  PRL_NATIVE_DECODE=$v timeout -k 10 300 python -u tools/loop_bench.py --model 1.5b --seq-length $S --samples-per-step 64 \
    --steps $N | grep '^{' | sed "s/}$/, \"native_decode\": $v}/" >> gpurun_out/ab_decode.jsonl
done
