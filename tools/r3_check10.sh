# Round 3, tenth GPU check: wider fixup iterations in the subset aggregation (parity suites, the
# subset bench and its kernel trace, the config-5 task).
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/r3c10
mkdir -p $O
cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest tests/test_gpu_subsets.py tests/test_gpu_config5.py -x -v --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || exit $?
timeout -k 10 300 python -u tools/bench_subsets.py --n 50000 > $O/bench_subsets.json 2> $O/bench_subsets.err || exit $?
timeout -k 10 600 python -u tools/bench_config5_task.py > $O/config5_task.json 2> $O/config5_task.err || exit $?
export TMPDIR=/tmp
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/sub_trace -o run -- \
    python3 $GRAFT_REPO_ROOT/tools/bench_subsets.py --n 50000 --groups 2 1000 > $O/sub_trace.json 2> $O/sub_trace.err
