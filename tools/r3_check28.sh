# Round 3: best-open fill with Iy opening from F = max(M, Ix) (default, shorter left-to-right chain)
# vs from B (libtaxi2_mi355x_yb.so): aligner suites on the default build, same-box A/B, then the
# profile of the default build (bench, rocprofv3 kernel trace + stats, PMC VALU / FETCH / WRITE).
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/r3c28
mkdir -p $O
cd $GRAFT_REPO_ROOT
timeout -k 10 700 python -u -m pytest tests/test_gpu_alignt.py tests/test_gpu_band.py tests/test_gpu_regress.py tests/test_gpu_parity.py tests/test_gpu_walk_strings.py -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || exit $?
for r in 1 2 3; do
  TAXI2_LIB=libtaxi2_mi355x_yb.so timeout -k 10 120 python -u bench.py --steps 8 --warmup 2 --no-cpu-baseline > $O/yb_$r.json 2> $O/yb_$r.err || exit $?
  timeout -k 10 120 python -u bench.py --steps 8 --warmup 2 --no-cpu-baseline > $O/yf_$r.json 2> $O/yf_$r.err || exit $?
done
PROF_NAME=r3c28/prof SKIP_PEAK=1 bash tools/profile_r2.sh > $O/profile.log 2>&1
