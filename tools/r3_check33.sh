# Round 3: other scores on the best-open fill (opens no better than extends) -- aligner and task
# suites, the guard build on the packed suites, then the scores bench with and without it
# (TAXI2_NO_BOPEN=1: the tagged sign-digit fill) and the default bench line.
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/r3c33
mkdir -p $O
cd $GRAFT_REPO_ROOT
PYT="python -u -m pytest -x -q --timeout 300 --timeout-method thread"
timeout -k 10 700 $PYT tests/test_gpu_alignt.py tests/test_gpu_band.py tests/test_gpu_regress.py tests/test_gpu_parity.py tests/test_gpu_walk_strings.py tests/test_gpu_long.py tests/test_gpu_tasks.py > $O/tests.log 2>&1 || exit $?
TAXI2_LIB=libtaxi2_mi355x_guard.so timeout -k 10 600 $PYT tests/test_gpu_alignt.py tests/test_gpu_regress.py tests/test_gpu_band.py > $O/tests_guard.log 2>&1 || exit $?
timeout -k 10 300 python -u tools/bench_scores.py > $O/scores_bopen.json 2> $O/scores_bopen.err || exit $?
TAXI2_NO_BOPEN=1 timeout -k 10 300 python -u tools/bench_scores.py > $O/scores_tagged.json 2> $O/scores_tagged.err || exit $?
timeout -k 10 120 python -u bench.py --steps 8 --warmup 2 --no-cpu-baseline > $O/bench.json 2> $O/bench.err
