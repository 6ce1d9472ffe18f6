# Round 3 (re-entry): HEAD after the two-stream aligned_pairs pipeline -- full GPU suite, smoke(),
# the default bench line, then the task bench at N = 5 000 / 10 000.
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/r3c24
mkdir -p $O
cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || exit $?
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit $?
timeout -k 10 300 python -u bench.py > $O/bench.json 2> $O/bench.err || exit $?
timeout -k 10 400 python -u tools/bench_task.py > $O/bench_task.json 2> $O/bench_task.err
