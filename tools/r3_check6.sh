# Round 3, sixth GPU check: chunked subset partials (parity suites incl. subsets wider than a
# chunk, config-5 exactness vs dense), subset bench, config 5 through VersusAll.start at full size,
# VersusAll.start() with the reference's defaults at N = 5 000 and 10 000 (outputs through
# /dev/null), then the HEAD profile of the headline kernel (tools/profile_r2.sh).
set -o pipefail
O=gpurun_out/r3c6
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_subsets.py tests/test_gpu_config5.py tests/test_gpu_streaming.py tests/test_gpu_walk_strings.py tests/test_gpu_tasks.py -x -v --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || exit $?
timeout -k 10 300 python -u tools/bench_subsets.py --n 50000 > $O/bench_subsets.json 2> $O/bench_subsets.err || exit $?
timeout -k 10 600 python -u tools/bench_config5_task.py > $O/config5_task.json 2> $O/config5_task.err || exit $?
timeout -k 10 900 python -u tools/bench_task.py > $O/bench_task.json 2> $O/bench_task.err || exit $?
PROF_NAME=prof_r3 SKIP_PEAK=1 bash tools/profile_r2.sh > $O/profile.log 2>&1
