#!/bin/bash
# PMC A/B of k_alignt2 builds / band widths on one box: for each NAME:LIB:BAND argument, one
# rocprofv3 --pmc pass (VALU / wave counters) over one bench launch.  Output: gpurun_out/pmc_ab/NAME/
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
export TMPDIR=/tmp
cd /tmp
for spec in "$@"; do
    name=${spec%%:*}; rest=${spec#*:}; lib=${rest%%:*}; band=${rest#*:}
    out=$R/gpurun_out/pmc_ab/$name
    mkdir -p $out
    TAXI2_LIB=$R/taxi2_amd/_lib/$lib TAXI2_AT_BAND=$band timeout -k 10 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE \
        --kernel-include-regex "k_alignt2" --output-format csv -d $out -o run -- \
        python3 $R/bench.py --steps 1 --warmup 0 --no-cpu-baseline > /dev/null 2> $out/err.txt || exit 1
done
