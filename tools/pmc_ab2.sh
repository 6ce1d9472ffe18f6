#!/bin/bash
# PMC A/B of packed-aligner builds on one box, two counter passes per build (one bench launch each):
#   A: VALU / wave-cycle split (SQ_WAIT_ANY + SQ_WAIT_INST_ANY + SQ_ACTIVE_INST_ANY ~= SQ_WAVE_CYCLES)
#   B: SALU / LDS instruction counts and LDS stalls
# Arguments NAME:LIB (band = capi.hip default).  Output: gpurun_out/pmc_ab2/NAME/{a,b}/
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
export TMPDIR=/tmp
cd /tmp
for spec in "$@"; do
    name=${spec%%:*}; lib=${spec#*:}
    out=$R/gpurun_out/pmc_ab2/$name
    mkdir -p $out
    TAXI2_LIB=$R/taxi2_amd/_lib/$lib timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE \
        --kernel-include-regex "k_alignt2" --output-format csv -d $out/a -o run -- \
        python3 $R/bench.py --steps 1 --warmup 0 --no-cpu-baseline > /dev/null 2> $out/a_err.txt || exit 1
    TAXI2_LIB=$R/taxi2_amd/_lib/$lib timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VMEM_WR SQ_BUSY_CYCLES GRBM_GUI_ACTIVE \
        --kernel-include-regex "k_alignt2" --output-format csv -d $out/b -o run -- \
        python3 $R/bench.py --steps 1 --warmup 0 --no-cpu-baseline > /dev/null 2> $out/b_err.txt || exit 1
done
