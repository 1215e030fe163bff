#!/bin/bash
# Dev: run one gpurun call, retrying (up to 8 times, 90 s apart) only when the GPU pool never ran the command
# (slots busy / box lost while being prepared / back-off) — never after the command itself ran.
# usage: tools/gpurun_retry.sh <out-file> <timeout-s> '<command>'
OUT=$1; TO=$2; CMD=$3
for i in 1 2 3 4 5 6 7 8; do
  /usr/local/graft/bin/gpurun --timeout "$TO" -- "$CMD" > "$OUT" 2>&1
  rc=$?
  if grep -q "slot(s) on this pod are busy\|stopped responding while being prepared\|taken away by the GPU service\|backing off\|no free box right now" "$OUT" && ! grep -q "status=ok" "$OUT"; then
    sleep 90; continue
  fi
  exit $rc
done
exit $rc
