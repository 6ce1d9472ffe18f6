# Round 3: the aligned form of config 5 through VersusAll.start (streamed triangle store, reductions
# only) at N = 20 000 (2.0e8 unordered pairs, 1 % of the full job), after the streaming suites.
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/r3c17
mkdir -p $O
cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest tests/test_gpu_streaming.py -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || exit $?
timeout -k 10 600 python -u tools/bench_config5_task.py --aligned --n 20000 > $O/config5_aligned_20000.json 2> $O/config5_aligned.err
