#!/bin/bash
# Run GPU steps in order, each under its own time limit; a step that fails its assertions (exit 1) lets
# the next one run, anything else (GPU fault / abort 134, segfault 139, timeout 124 / 137, hang) ends the call.
# usage: tools/gpu_steps.sh "<seconds>|<log>|<command>" ...
for spec in "$@"; do
  secs="${spec%%|*}"; rest="${spec#*|}"; log="${rest%%|*}"; cmd="${rest#*|}"
  echo "[step] $cmd  (limit ${secs}s, log $log)"
  timeout -k 10 "$secs" bash -c "$cmd" > "$log" 2>&1
  rc=$?
  echo "[step] rc=$rc"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "[step] stopping: rc=$rc"; exit $rc; fi
done
exit 0
