# Round 3, eleventh GPU check: aligned_pairs.txt from one fill per unordered pair (tri strings +
# pointer text), parity against the rect path and the task suites, then the task bench.
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/r3c11
mkdir -p $O
cd $GRAFT_REPO_ROOT
timeout -k 10 700 python -u -m pytest tests/test_gpu_walk_strings.py tests/test_gpu_tasks.py tests/test_gpu_streaming.py tests/test_writers_native.py -x -v --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || exit $?
timeout -k 10 700 python -u tools/bench_task.py > $O/bench_task.json 2> $O/bench_task.err
