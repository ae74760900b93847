# rocprofv3 kernel stats of a command; keeps only the *_stats.csv summaries under gpurun_out/<name>
#   bash tools/prof_stats.sh <name> <seconds> <python args...>
name=$1; secs=$2; shift 2
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 "$secs" rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/prof_$name -o run -- python3 "$@" > gpurun_out/$name.log 2>&1
rc=$?
mkdir -p gpurun_out/$name
find /tmp/prof_$name -name "*_stats.csv" -exec cp {} gpurun_out/$name/ \;
exit $rc
