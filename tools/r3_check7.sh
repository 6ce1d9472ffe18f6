# Round 3, seventh GPU check: pinned aligned-pairs text + larger string-emitting row blocks (task
# suites), VersusAll.start() with the reference's defaults at N = 5 000 / 10 000, then the HEAD
# profile of the headline kernel (tools/profile_r2.sh: bench, kernel trace, VALU / FETCH / WRITE).
set -o pipefail
O=gpurun_out/r3c7
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_walk_strings.py tests/test_gpu_streaming.py tests/test_gpu_tasks.py -x -v --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || exit $?
timeout -k 10 700 python -u tools/bench_task.py > $O/bench_task.json 2> $O/bench_task.err || exit $?
PROF_NAME=prof_r3 SKIP_PEAK=1 bash tools/profile_r2.sh > $O/profile.log 2>&1
