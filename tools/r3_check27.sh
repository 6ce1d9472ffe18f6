# Round 3: best-open fill -- the poisoning guard build on the packed-aligner suites, a same-box A/B
# of the out-of-band skip on the new fill, then the profile of the default build (bench line,
# rocprofv3 kernel trace + stats, PMC passes: VALU, FETCH_SIZE, WRITE_SIZE).
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/r3c27
mkdir -p $O
cd $GRAFT_REPO_ROOT
PYT="python -u -m pytest -x -q --timeout 300 --timeout-method thread"
TAXI2_LIB=libtaxi2_mi355x_guard.so timeout -k 10 600 $PYT tests/test_gpu_alignt.py tests/test_gpu_regress.py tests/test_gpu_band.py > $O/tests_guard.log 2>&1 || exit $?
for r in 1 2; do
  timeout -k 10 120 python -u bench.py --steps 8 --warmup 2 --no-cpu-baseline > $O/main_$r.json 2> $O/main_$r.err || exit $?
  TAXI2_LIB=libtaxi2_mi355x_skip.so timeout -k 10 120 python -u bench.py --steps 8 --warmup 2 --no-cpu-baseline > $O/skip_$r.json 2> $O/skip_$r.err || exit $?
done
TAXI2_LIB=libtaxi2_mi355x_skip.so timeout -k 10 600 $PYT tests/test_gpu_alignt.py tests/test_gpu_band.py > $O/tests_skip.log 2>&1 || exit $?
PROF_NAME=r3c27/prof SKIP_PEAK=1 bash tools/profile_r2.sh > $O/profile.log 2>&1
