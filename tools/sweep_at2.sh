#!/bin/bash
# Bench the trace-and-walk aligners (packed default and 32-bit) over chunk sizes (GPU box).
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/sweep_at2.log
: > $OUT
for mode in packed t32; do
  for chunk in ${CHUNKS:-8 6}; do
    env=""
    [ $mode = t32 ] && env="TAXI2_NO_PACKED=1"
    r=$(env $env TAXI2_AT_CHUNK=$chunk timeout -k 10 120 python3 $R/bench.py --steps 2 --warmup 1 --no-cpu-baseline 2>/dev/null) || { echo "$mode chunk=$chunk FAILED" >> $OUT; exit 1; }
    v=$(echo "$r" | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["value"]), round(d["roofline"]["kernel_ms"],1))')
    echo "$mode chunk=$chunk $v" >> $OUT
  done
done
cat $OUT
