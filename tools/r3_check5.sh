# Round 3, fifth GPU check: the full GPU suite on the new defaults (always-encode packed aligner,
# multi-grid subset partials), the default bench line, the subset-aggregation bench, config 5
# through VersusAll.start at full size, and a kernel trace of bench.py (CSV stats).
set -o pipefail
O=gpurun_out/r3c5
mkdir -p $O
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || exit $?
timeout -k 10 300 python -u bench.py > $O/bench.json 2> $O/bench.err || exit $?
timeout -k 10 300 python -u tools/bench_subsets.py --n 50000 > $O/bench_subsets.json 2> $O/bench_subsets.err || exit $?
timeout -k 10 600 python -u tools/bench_config5_task.py > $O/config5_task.json 2> $O/config5_task.err || exit $?
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_bench -o bench -- python3 -u bench.py --steps 5 --warmup 1 --no-cpu-baseline > $O/prof_bench.json 2> $O/prof_bench.err
