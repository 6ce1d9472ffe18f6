# Round 3 end-of-session HEAD check: the full GPU suite, smoke, then the profiling recipe
# (bench line with the CPU baseline, rocprofv3 kernel trace + stats, VALU / FETCH / WRITE PMC passes).
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/r3c36
mkdir -p $O
cd $GRAFT_REPO_ROOT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || exit $?
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit $?
SKIP_PEAK=1 PROF_NAME=r3c36/prof bash tools/profile_r2.sh
