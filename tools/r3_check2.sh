# Round 3, second GPU check: exact parallel subset aggregation, tiled pre-aligned kernel, walker
# strings, streamed paths (single and 2-rank sharded), task outputs, config 5 through the task path.
set -o pipefail
O=gpurun_out/r3c2
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_gpu_subsets.py tests/test_gpu_prealigned.py tests/test_gpu_walk_strings.py tests/test_gpu_streaming.py tests/test_gpu_tasks.py -x -v --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || exit $?
timeout -k 10 600 python -u tools/bench_config5_task.py > $O/config5_task.json 2> $O/config5_task.err || exit $?
timeout -k 10 900 python -u -m pytest tests/test_gpu_config5.py -x -v -s --timeout 900 --timeout-method thread > $O/config5_test.log 2>&1
