# Round 3: best-open fill (four maxima per cell pair, D1 = M - Ix / D2 = M - Iy trace) -- the
# aligner parity suites on the new build, then a same-box bench A/B against the previous build.
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/r3c26
mkdir -p $O
cd $GRAFT_REPO_ROOT
timeout -k 10 700 python -u -m pytest tests/test_gpu_alignt.py tests/test_gpu_band.py tests/test_gpu_regress.py tests/test_gpu_parity.py tests/test_gpu_walk_strings.py -x -v --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || exit $?
for r in 1 2; do
  TAXI2_LIB=libtaxi2_mi355x_r3old.so timeout -k 10 120 python -u bench.py --steps 8 --warmup 2 --no-cpu-baseline > $O/old_$r.json 2> $O/old_$r.err || exit $?
  timeout -k 10 120 python -u bench.py --steps 8 --warmup 2 --no-cpu-baseline > $O/new_$r.json 2> $O/new_$r.err || exit $?
done
