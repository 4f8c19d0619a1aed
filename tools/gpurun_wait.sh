#!/bin/bash
# Waits for a free GPU box: re-submits the same command only while gpurun
# reports that no box was free or that it is backing off (nothing ran,
# nothing charged), sleeping as long as it asks; any other outcome (success,
# failure, refusal) ends the loop at once.
#   tools/gpurun_wait.sh <timeout-seconds> <command> [max-tries]
t=$1; cmd=$2; tries=${3:-30}
for i in $(seq 1 "$tries"); do
  out=$(/usr/local/graft/bin/gpurun --timeout "$t" -- "$cmd" 2>&1); rc=$?
  echo "$out" | tail -4
  if echo "$out" | grep -q "status=transient"; then
    s=$(echo "$out" | grep -o "retry in [0-9]*s" | grep -o "[0-9]*" | head -1)
    sleep $(( ${s:-150} + 10 ))
    continue
  fi
  exit $rc
done
exit 3
