#!/bin/bash
# Run a sequence of GPU steps on the gpurun box; stop at the first step that faults, aborts,
# segfaults or times out (exit 124/134/137/139 or >128). A plain test failure (exit 1) does not stop
# later steps. Usage: tools/gpu_session.sh "<name>:<timeout>:<cmd>" ...
mkdir -p gpurun_out
export TMPDIR=/tmp
for spec in "$@"; do
  name="${spec%%:*}"; rest="${spec#*:}"; to="${rest%%:*}"; cmd="${rest#*:}"
  echo "=== [$name] (timeout ${to}s) $cmd" | tee -a gpurun_out/session.log
  start=$(date +%s)
  timeout -k 10 "$to" bash -c "$cmd" > "gpurun_out/$name.log" 2>&1
  rc=$?
  echo "=== [$name] rc=$rc in $(( $(date +%s) - start ))s" | tee -a gpurun_out/session.log
  tail -n 25 "gpurun_out/$name.log"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ] && [ $rc -ne 2 ] && [ $rc -ne 5 ]; then
    echo "=== stopping: step $name ended with rc=$rc" | tee -a gpurun_out/session.log
    exit $rc
  fi
done
