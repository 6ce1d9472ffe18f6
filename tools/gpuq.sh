#!/bin/bash
# usage: tools/gpuq.sh LOG 'command' -- one gpurun call, re-queued only while gpurun reports that no box
# or slot was available (exit code 3: nothing ran, nothing charged); any other outcome is final
LOG=$1; shift
for i in $(seq 1 40); do
  timeout 2400 /usr/local/graft/bin/gpurun --timeout 1200 -- "$@" > "$LOG" 2>&1
  rc=$?
  if [ $rc -eq 3 ]; then sleep 60; continue; fi
  echo "rc=$rc" >> "$LOG"; exit $rc
done
