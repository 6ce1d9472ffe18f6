# Round 3: same-box A/B of A2_MNEXT=2 against A2_MNEXT=1 + A2_MNEXT_WAIT=1 (next-column M ordering on
# both fill waves, vector memory drained before the last wave's step loop), alternating; the aligner
# parity suites on the mw build.
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/r3c38
mkdir -p $O
cd $GRAFT_REPO_ROOT
for r in 1 2 3; do
  for L in mnext2 mw; do
    N=${L:-def}
    TAXI2_LIB=libtaxi2_mi355x${L:+_$L}.so timeout -k 10 150 python -u bench.py --steps 8 --warmup 2 --no-cpu-baseline > $O/${N}_$r.json 2> $O/${N}_$r.err || exit $?
  done
done
TAXI2_LIB=libtaxi2_mi355x_mw.so timeout -k 10 900 python -u -m pytest tests/test_gpu_alignt.py tests/test_gpu_regress.py tests/test_gpu_band.py tests/test_gpu_parity.py tests/test_gpu_walk_strings.py -x -q --timeout 300 --timeout-method thread > $O/tests_mw.log 2>&1
