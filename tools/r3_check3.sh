# Round 3, third GPU check: new parity suites (subsets, tiled pre-aligned, walker strings, streaming
# incl. duplicate ids / wide / 2-rank sharded reductions, task outputs), A/B of the skip vs no-skip
# raw-difference build, config 5 through the task path.
set -o pipefail
O=gpurun_out/r3c3
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_gpu_subsets.py tests/test_gpu_prealigned.py tests/test_gpu_walk_strings.py tests/test_gpu_streaming.py tests/test_gpu_tasks.py tests/test_gpu_ncd.py -x -v --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || exit $?
for r in 1 2; do
  timeout -k 10 150 python -u bench.py --steps 8 --warmup 2 --no-cpu-baseline > $O/main_$r.json 2> $O/main_$r.err || exit $?
  TAXI2_LIB=libtaxi2_mi355x_noskip.so timeout -k 10 150 python -u bench.py --steps 8 --warmup 2 --no-cpu-baseline > $O/noskip_$r.json 2> $O/noskip_$r.err || exit $?
done
timeout -k 10 600 python -u tools/bench_config5_task.py > $O/config5_task.json 2> $O/config5_task.err || exit $?
timeout -k 10 900 python -u -m pytest tests/test_gpu_config5.py -x -v -s --timeout 900 --timeout-method thread > $O/config5_test.log 2>&1
