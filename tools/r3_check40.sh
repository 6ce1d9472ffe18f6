# Round 3 HEAD check after the maximum3 fill: the full GPU suite, the poisoning guard build on the
# packed aligner suites, smoke, then the profiling recipe (bench line with the CPU baseline,
# rocprofv3 kernel trace + stats, the VALU issue microbenchmark, VALU / FETCH / WRITE PMC passes).
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/r3c40
mkdir -p $O
cd $GRAFT_REPO_ROOT
PYT="python -u -m pytest -x -q --timeout 300 --timeout-method thread"
timeout -k 10 900 $PYT tests -m gpu > $O/tests.log 2>&1 || exit $?
TAXI2_LIB=libtaxi2_mi355x_guard.so timeout -k 10 600 $PYT tests/test_gpu_alignt.py tests/test_gpu_regress.py tests/test_gpu_band.py > $O/tests_guard.log 2>&1 || exit $?
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit $?
PROF_NAME=r3c40/prof bash tools/profile_r2.sh
