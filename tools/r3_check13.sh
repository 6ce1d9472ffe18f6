# Round 3, thirteenth GPU check: the full GPU suite, smoke() and the default bench line on HEAD.
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/r3c13
mkdir -p $O
cd $GRAFT_REPO_ROOT
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || exit $?
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit $?
timeout -k 10 300 python -u bench.py > $O/bench.json 2> $O/bench.err
