# Round 3 re-entry HEAD check: full GPU suite, smoke, the default bench line (with the CPU
# baseline) and a kernel trace of bench.py (CSV stats) on the HEAD build.
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/r3c34
mkdir -p $O
cd $GRAFT_REPO_ROOT
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || exit $?
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit $?
timeout -k 10 400 python -u bench.py > $O/bench.json 2> $O/bench.err || exit $?
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_bench -o bench -- python3 -u bench.py --steps 5 --warmup 1 --no-cpu-baseline > $O/prof_bench.json 2> $O/prof_bench.err
