# Round 3: same-box A/B of HEAD (base), the 24-bit row-score word alone (oyonly, A2_MNEXT=0) and
# both changes (the default build: next-column M formed before the new B), alternating; then the
# aligner parity suites on the default build.
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/r3c35
mkdir -p $O
cd $GRAFT_REPO_ROOT
for r in 1 2; do
  for L in base oyonly ""; do
    N=${L:-new}
    TAXI2_LIB=libtaxi2_mi355x${L:+_$L}.so timeout -k 10 150 python -u bench.py --steps 8 --warmup 2 --no-cpu-baseline > $O/${N}_$r.json 2> $O/${N}_$r.err || exit $?
  done
done
timeout -k 10 900 python -u -m pytest tests/test_gpu_alignt.py tests/test_gpu_regress.py tests/test_gpu_band.py tests/test_gpu_parity.py tests/test_gpu_walk_strings.py -x -q --timeout 300 --timeout-method thread > $O/tests_new.log 2>&1
