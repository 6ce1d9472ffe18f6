# Round 3: branch-free best-open walker (walk_run_raw) -- aligner suites, then a same-box A/B
# against the best-open build with the branchy walker (yb).
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/r3c31
mkdir -p $O
cd $GRAFT_REPO_ROOT
timeout -k 10 700 python -u -m pytest tests/test_gpu_alignt.py tests/test_gpu_band.py tests/test_gpu_regress.py tests/test_gpu_parity.py tests/test_gpu_walk_strings.py -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || exit $?
for r in 1 2 3; do
  TAXI2_LIB=libtaxi2_mi355x_yb.so timeout -k 10 120 python -u bench.py --steps 8 --warmup 2 --no-cpu-baseline > $O/yb_$r.json 2> $O/yb_$r.err || exit $?
  timeout -k 10 120 python -u bench.py --steps 8 --warmup 2 --no-cpu-baseline > $O/bf_$r.json 2> $O/bf_$r.err || exit $?
done
