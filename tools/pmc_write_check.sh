#!/bin/bash
# Spill check: WRITE_SIZE / FETCH_SIZE (separate passes) of the single-orientation kernels for the
# variants given as arguments (TAXI2_VARIANT1 shapes), one bench launch each.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd /tmp; export TMPDIR=/tmp
for v in "$@"; do
  for c in WRITE_SIZE FETCH_SIZE; do
    TAXI2_VARIANT1=$v timeout -k 10 200 rocprofv3 --pmc $c --kernel-include-regex "k_align1" --output-format csv \
      -d $R/gpurun_out/pmc_${c}_$v -o run -- python3 $R/bench.py --steps 1 --warmup 0 --no-cpu-baseline \
      > /dev/null 2> $R/gpurun_out/pmc_${c}_$v.err || exit 1
  done
done
