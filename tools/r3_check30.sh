# Round 3: best-open fill with the uniform Ix-open constant in the cell loop (no early update) --
# aligner suites on the default build, same-box A/B against B-open without it (yb) and with the LDS
# half-word substitution reads (d16), then the profile of the default build.
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/r3c30
mkdir -p $O
cd $GRAFT_REPO_ROOT
timeout -k 10 700 python -u -m pytest tests/test_gpu_alignt.py tests/test_gpu_band.py tests/test_gpu_regress.py tests/test_gpu_parity.py tests/test_gpu_walk_strings.py -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || exit $?
for r in 1 2; do
  TAXI2_LIB=libtaxi2_mi355x_yb.so timeout -k 10 120 python -u bench.py --steps 8 --warmup 2 --no-cpu-baseline > $O/yb_$r.json 2> $O/yb_$r.err || exit $?
  timeout -k 10 120 python -u bench.py --steps 8 --warmup 2 --no-cpu-baseline > $O/main_$r.json 2> $O/main_$r.err || exit $?
  TAXI2_LIB=libtaxi2_mi355x_d16.so timeout -k 10 120 python -u bench.py --steps 8 --warmup 2 --no-cpu-baseline > $O/d16_$r.json 2> $O/d16_$r.err || exit $?
done
TAXI2_LIB=libtaxi2_mi355x_d16.so timeout -k 10 600 python -u -m pytest tests/test_gpu_alignt.py tests/test_gpu_band.py -x -q --timeout 300 --timeout-method thread > $O/tests_d16.log 2>&1 || exit $?
PROF_NAME=r3c30/prof SKIP_PEAK=1 bash tools/profile_r2.sh > $O/profile.log 2>&1
