#!/bin/bash
# One runner for every GPU-box job of this repo (replaces round 1-3's one-off check scripts).
#   gpurun --timeout 1200 -- 'bash tools/gpu_run.sh TAG STEP [STEP ...]'
# Outputs go to gpurun_out/TAG/.  Each STEP runs under its own time limit; the steps are chained
# and the runner stops at the first failure (no GPU step after a fault, abort or timeout).
# Steps:
#   suite            python -m pytest tests -m gpu (the driver's round-end command)
#   tests:F1,F2      those test files only (tests/F.py), e.g. tests:test_gpu_alignt,test_gpu_band
#   smoke            __graft_entry__.smoke()
#   bench            bench.py (default settings: headline + secondary legs)
#   headline         bench.py --secondary '' --steps 10 --warmup 2
#   ab:LIBA,LIBB,R   R alternations of the headline with TAXI2_LIB=LIBA then LIBB (same box A/B)
#   abenv:VAR,R      R alternations of the headline with VAR=1 set, then unset (same box A/B)
#   hl:NAME:V=X,...  one headline run with those environment settings -> hl_NAME.json / .err
#   trace            rocprofv3 --kernel-trace --stats of the headline bench
#   pmc_valu | pmc_fetch | pmc_write | pmc_lds
#                    one rocprofv3 --pmc pass each over one bench launch (separate runs: rocprofv3
#                    does not split counters over passes)
#   guard            the poisoning guard build (make guard) on the packed aligner suites
#   peak             tools/valu_peak (SIMD cycles per wave64 instruction)
#   d2h              tools/d2h_probe (device -> host text bandwidth: memcpy, 4 streams, kernel stores)
#   tool:SCRIPT      python tools/SCRIPT.py (bench tools), e.g. tool:bench_long
#   tooltrace:SCRIPT rocprofv3 --kernel-trace --stats of that tool
#   sec:LEG          one bench_secondary.py leg alone (task, config5, config4, allmetrics)
#   with:V=X,...:STEP  any step with those environment settings (outputs under the step's own names)
#   secenv:NAME:LEG:V=X,...  that leg with those environment settings -> secenv_NAME.json
#   sectrace:LEG     rocprofv3 --kernel-trace --stats of that leg
#   pmcsec:LEG:SET   one rocprofv3 --pmc pass (valu | lds | fetch | write) over that leg's kernels
#                    matching PMC_SEC_RE (default k_prealigned|k_subset|k_rowmin)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:?tag}
shift
OUT=$R/gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
PYT="python -u -m pytest -x -v --timeout 300 --timeout-method thread"
BENCH="python3 $R/bench.py --secondary= --no-cpu-baseline"
PMC_OPTS="--kernel-include-regex k_align --output-format csv"
# the library's baked-in source hash beside the tree's, first line of every test log
BUILD_LINE="from taxi2_amd._native import build_info; print('engine build:', build_info())"

run_step() {
    local s=$1
    case "$s" in
    suite)
        (cd "$R" && python3 -c "$BUILD_LINE" > "$OUT/suite.log" 2>&1 && \
            timeout -k 10 1000 $PYT tests -m gpu >> "$OUT/suite.log" 2>&1) ;;
    tests:*)
        local files=""
        for f in $(echo "${s#tests:}" | tr ',' ' '); do files="$files tests/$f.py"; done
        local log="$OUT/tests_$(echo "${s#tests:}" | tr ',' '_').log"
        (cd "$R" && python3 -c "$BUILD_LINE" > "$log" 2>&1 && timeout -k 10 900 $PYT $files >> "$log" 2>&1) ;;
    smoke)
        (cd "$R" && timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1) ;;
    bench)
        (cd "$R" && timeout -k 10 600 python3 -u bench.py > "$OUT/bench.json" 2> "$OUT/bench.err") ;;
    headline)
        (cd "$R" && timeout -k 10 300 python3 -u bench.py --secondary= --steps 10 --warmup 2 > "$OUT/headline.json" 2> "$OUT/headline.err") ;;
    ab:*)
        IFS=, read -r la lb reps <<< "${s#ab:}"
        for r in $(seq 1 "${reps:-2}"); do
            (cd "$R" && TAXI2_LIB=$la timeout -k 10 200 $BENCH --steps 8 --warmup 2 > "$OUT/ab_${la%.so}_$r.json" 2> "$OUT/ab_${la%.so}_$r.err") || return $?
            (cd "$R" && TAXI2_LIB=$lb timeout -k 10 200 $BENCH --steps 8 --warmup 2 > "$OUT/ab_${lb%.so}_$r.json" 2> "$OUT/ab_${lb%.so}_$r.err") || return $?
        done ;;
    abenv:*)
        IFS=, read -r var reps <<< "${s#abenv:}"
        for r in $(seq 1 "${reps:-2}"); do
            (cd "$R" && env "$var=1" timeout -k 10 200 $BENCH --steps 8 --warmup 2 > "$OUT/ab_env_$r.json" 2> "$OUT/ab_env_$r.err") || return $?
            (cd "$R" && timeout -k 10 200 $BENCH --steps 8 --warmup 2 > "$OUT/ab_def_$r.json" 2> "$OUT/ab_def_$r.err") || return $?
        done ;;
    hl:*)
        local rest=${s#hl:}
        local name=${rest%%:*}
        local envs=$(echo "${rest#*:}" | tr ',' ' ')
        (cd "$R" && env $envs timeout -k 10 200 $BENCH --steps 8 --warmup 2 > "$OUT/hl_$name.json" 2> "$OUT/hl_$name.err") ;;
    trace)
        (cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace" -o run -- \
            $BENCH --steps 10 --warmup 2 > "$OUT/trace_bench.json" 2> "$OUT/trace.err") ;;
    pmc_valu)
        (cd /tmp && timeout -s KILL 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY \
            SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE $PMC_OPTS -d "$OUT/pmc_valu" -o run -- \
            $BENCH --steps 1 --warmup 0 > /dev/null 2> "$OUT/pmc_valu.err") ;;
    pmc_lds)
        (cd /tmp && timeout -s KILL 300 rocprofv3 --pmc SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_ANY SQ_INSTS_SALU SQ_INSTS_VMEM \
            SQ_INST_CYCLES_VMEM GRBM_GUI_ACTIVE $PMC_OPTS -d "$OUT/pmc_lds" -o run -- \
            $BENCH --steps 1 --warmup 0 > /dev/null 2> "$OUT/pmc_lds.err") ;;
    pmc_mem)  # the vector-memory and texture pipeline: instruction counts and TA/TD busy
        (cd /tmp && timeout -s KILL 300 rocprofv3 --pmc SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_FLAT SQ_INSTS_SMEM \
            TA_TA_BUSY_sum TA_BUFFER_WAVEFRONTS_sum GRBM_GUI_ACTIVE $PMC_OPTS -d "$OUT/pmc_mem" -o run -- \
            $BENCH --steps 1 --warmup 0 > /dev/null 2> "$OUT/pmc_mem.err") ;;
    pmc_fetch)
        (cd /tmp && timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE $PMC_OPTS -d "$OUT/pmc_fetch" -o run -- \
            $BENCH --steps 1 --warmup 0 > /dev/null 2> "$OUT/pmc_fetch.err") ;;
    pmc_write)
        (cd /tmp && timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE $PMC_OPTS -d "$OUT/pmc_write" -o run -- \
            $BENCH --steps 1 --warmup 0 > /dev/null 2> "$OUT/pmc_write.err") ;;
    pmcsec:*)  # pmcsec:LEG:SET -- one PMC pass (SET valu | lds | fetch | write) over a bench_secondary leg,
        # kernels matching PMC_SEC_RE (default: the pre-aligned tile and subset kernels)
        local rest=${s#pmcsec:}
        local leg=${rest%%:*} set=${rest#*:}
        local re=${PMC_SEC_RE:-k_prealigned|k_subset|k_rowmin}
        local ctr
        case "$set" in
            valu) ctr="SQ_WAVES SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE" ;;
            lds) ctr="SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_ANY SQ_INSTS_SALU SQ_INSTS_VMEM SQ_INST_CYCLES_VMEM GRBM_GUI_ACTIVE" ;;
            fetch) ctr="FETCH_SIZE" ;;
            write) ctr="WRITE_SIZE" ;;
            *) echo "unknown pmc set $set" >&2; return 2 ;;
        esac
        # (the prealigned leg: config 5's tile launches alone, TAXI2_PREALIGNED_PARTS=config5)
        (cd /tmp && TAXI2_PREALIGNED_PARTS=config5 timeout -s KILL 400 rocprofv3 --pmc $ctr --kernel-include-regex "$re" \
            --output-format csv -d "$OUT/pmcsec_${leg}_$set" -o run -- python3 $R/bench_secondary.py "$leg" \
            > "$OUT/pmcsec_${leg}_$set.json" 2> "$OUT/pmcsec_${leg}_$set.err") ;;
    guard)
        (cd "$R" && TAXI2_LIB=libtaxi2_mi355x_guard.so timeout -k 10 900 $PYT tests/test_gpu_alignt.py \
            tests/test_gpu_band.py tests/test_gpu_regress.py > "$OUT/guard.log" 2>&1) ;;
    peak)
        timeout -k 10 180 "$R/tools/valu_peak" > "$OUT/valu_peak.txt" 2>&1 ;;
    d2h)
        timeout -k 10 120 "$R/tools/d2h_probe" > "$OUT/d2h_probe.txt" 2>&1 ;;
    tool:*)
        (cd "$R" && timeout -k 10 900 python3 -u "tools/${s#tool:}.py" > "$OUT/${s#tool:}.json" 2> "$OUT/${s#tool:}.err") ;;
    tooltrace:*)  # rocprofv3 --kernel-trace --stats of python tools/SCRIPT.py
        (cd /tmp && timeout -k 10 900 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/tooltrace_${s#tooltrace:}" -o run -- \
            python3 "$R/tools/${s#tooltrace:}.py" > "$OUT/tooltrace_${s#tooltrace:}.json" 2> "$OUT/tooltrace_${s#tooltrace:}.err") ;;
    sec:*)
        # (sec:A+B+C: those legs one after another in one process, as bench.py runs them)
        (cd "$R" && timeout -k 10 600 python3 -u bench_secondary.py $(echo "${s#sec:}" | tr '+' ' ') > "$OUT/sec_${s#sec:}.json" 2> "$OUT/sec_${s#sec:}.err") ;;
    with:*)  # with:V=X,...:STEP -- any other step with those environment settings
        local rest=${s#with:}
        local envs=${rest%%:*} inner=${rest#*:}
        (for kv in $(echo "$envs" | tr ',' ' '); do export "$kv"; done; run_step "$inner") ;;
    secenv:*)  # secenv:NAME:LEG:V=X,... -- one bench_secondary leg with those environment settings
        local rest=${s#secenv:}
        local name=${rest%%:*}; rest=${rest#*:}
        local leg=${rest%%:*} envs=${rest#*:}
        (cd "$R" && env $(echo "$envs" | tr ',' ' ') timeout -k 10 600 python3 -u bench_secondary.py $(echo "$leg" | tr '+' ' ') \
            > "$OUT/secenv_$name.json" 2> "$OUT/secenv_$name.err") ;;
    sectrace:*)
        (cd /tmp && timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/sectrace_${s#sectrace:}" -o run -- \
            python3 $R/bench_secondary.py "${s#sectrace:}" > "$OUT/sectrace_${s#sectrace:}.json" 2> "$OUT/sectrace_${s#sectrace:}.err") ;;
    *)
        echo "unknown step $s" >&2; return 2 ;;
    esac
}

for s in "$@"; do
    echo "[gpu_run $TAG] $s" >&2
    run_step "$s"
    rc=$?
    echo "[gpu_run $TAG] $s rc=$rc" >&2
    if [ $rc -ne 0 ]; then
        exit $rc
    fi
done
