# Round 3 end: the packed aligner suite with the maximum3 value-range extremes test, then configs 2 /
# 4 (65 536-query slice) / 5 and the default versusAll task at N = 5 000 on the HEAD build.
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/r3c42
mkdir -p $O
cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest tests/test_gpu_alignt.py -x -v --timeout 300 --timeout-method thread > $O/tests_alignt.log 2>&1 &&
timeout -k 10 300 python -u tools/bench_configs.py --config2 --config5 > $O/configs.json 2> $O/configs.err &&
timeout -k 10 400 python -u tools/bench_configs.py --config4 --q-slice 65536 --steps 1 > $O/config4_65536.json 2> $O/config4.err &&
timeout -k 10 300 python -u tools/bench_task.py --n 5000 > $O/task_5000.json 2> $O/task.err
