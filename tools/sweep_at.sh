#!/bin/bash
# Sweep the trace-and-walk aligner's launch knobs on the bench workload (run on the GPU box).
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/sweep_at.log
: > $OUT
for chunk in ${CHUNKS:-8 4 6}; do
  for hops in ${HOPS:-8 16 32 64}; do
    r=$(TAXI2_AT_CHUNK=$chunk TAXI2_AT_HOPS=$hops timeout -k 10 120 python3 $R/bench.py --steps 2 --warmup 1 --no-cpu-baseline 2>/dev/null) || { echo "chunk=$chunk hops=$hops FAILED" >> $OUT; exit 1; }
    v=$(echo "$r" | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["value"]), round(d["roofline"]["kernel_ms"],1))')
    echo "chunk=$chunk hops=$hops $v" >> $OUT
  done
done
cat $OUT
