#!/usr/bin/env bash
# Run GPU steps in order, each under its own time limit.  An ordinary failure (exit 1, e.g. a
# failing test) lets later steps run; a crash / abort / timeout (124 125 134 137 139, or a
# signal) ends the session: nothing else touches the GPU after that.
#   tools/gpu_session.sh "name:seconds:command" ...
set -u
mkdir -p gpurun_out
for spec in "$@"; do
  name="${spec%%:*}"; rest="${spec#*:}"; secs="${rest%%:*}"; cmd="${rest#*:}"
  echo "=== [$name] (limit ${secs}s): $cmd" | tee -a gpurun_out/session.log
  start=$(date +%s)
  timeout -k 10 "$secs" bash -c "$cmd" > "gpurun_out/$name.log" 2>&1
  rc=$?
  echo "=== [$name] rc=$rc after $(( $(date +%s) - start ))s" | tee -a gpurun_out/session.log
  tail -n 25 "gpurun_out/$name.log"
  case $rc in
    0|1|2|5) ;;
    *) echo "=== stopping: step $name ended with rc=$rc" | tee -a gpurun_out/session.log; exit $rc ;;
  esac
done
