#!/bin/bash
# Profiling recipe (run on the GPU box from the repo root; PROF_NAME names the output dir):
#   0. tools/valu_peak (VALU issue ceiling of the aligner's instructions, 1..8 waves per SIMD)
#   1. bench line (default settings)
#   2. rocprofv3 --kernel-trace --stats of the same bench command
#   3. separate --pmc passes over one launch: VALU / wave activity; FETCH_SIZE; WRITE_SIZE
# Every GPU step has its own time limit; steps are chained with && (stop at the first failure).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/${PROF_NAME:-prof_r2}
mkdir -p $OUT
export TMPDIR=/tmp
cd /tmp
step0() {
    if [ -n "$SKIP_PEAK" ]; then return 0; fi
    timeout -k 10 180 $R/tools/valu_peak > $OUT/valu_peak.txt 2>&1
}
step0 &&
timeout -k 10 420 python3 $R/bench.py --steps 10 --warmup 2 > $OUT/bench.json 2> $OUT/bench.err &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- \
    python3 $R/bench.py --steps 10 --warmup 2 --no-cpu-baseline > $OUT/trace_bench.json 2> $OUT/trace.err &&
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE \
    --kernel-include-regex "k_align" --output-format csv -d $OUT/pmc_valu -o run -- \
    python3 $R/bench.py --steps 1 --warmup 0 --no-cpu-baseline > /dev/null 2> $OUT/pmc_valu.err &&
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex "k_align" --output-format csv -d $OUT/pmc_fetch -o run -- \
    python3 $R/bench.py --steps 1 --warmup 0 --no-cpu-baseline > /dev/null 2> $OUT/pmc_fetch.err &&
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex "k_align" --output-format csv -d $OUT/pmc_write -o run -- \
    python3 $R/bench.py --steps 1 --warmup 0 --no-cpu-baseline > /dev/null 2> $OUT/pmc_write.err
rc=$?
echo "profile rc=$rc"
find $OUT -name "*.csv" | head -20
exit $rc
