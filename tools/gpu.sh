#!/bin/bash
# Host-side helper: submit ONE gpurun call; resubmit only when the infrastructure reports that
# nothing ran (status=transient / back-off / exit 3).  A command that ran and failed is never retried.
# usage: tools/gpu.sh <timeout_s> '<command>'
T=$1; shift
for i in 1 2 3 4 5 6 7 8; do
  out=$(/usr/local/graft/bin/gpurun --timeout "$T" -- "$@" 2>&1); rc=$?
  echo "$out" | tail -4
  if echo "$out" | grep -q "status=transient\|backing off" || [ $rc -eq 3 ]; then
    w=$(echo "$out" | grep -o "retry in [0-9]*s" | grep -o "[0-9]*"); sleep $(( ${w:-30} + 20 )); continue
  fi
  exit $rc
done
exit 3
