# Round 3, eighth GPU check: natural-order subset rows for few subsets (parity: both row paths,
# config-5 exactness vs dense), subset bench, config-5 task, default bench line (compute roofline
# now also against the full-rate ceiling).
set -o pipefail
O=gpurun_out/r3c8
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_subsets.py tests/test_gpu_config5.py tests/test_gpu_streaming.py -x -v --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || exit $?
timeout -k 10 300 python -u tools/bench_subsets.py --n 50000 > $O/bench_subsets.json 2> $O/bench_subsets.err || exit $?
timeout -k 10 600 python -u tools/bench_config5_task.py > $O/config5_task.json 2> $O/config5_task.err || exit $?
timeout -k 10 300 python -u bench.py > $O/bench.json 2> $O/bench.err
