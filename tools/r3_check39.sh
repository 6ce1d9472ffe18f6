# Round 3: same-box A/B of HEAD (head) against A2_MAX3 (bias 20480, the default-score best-open
# fill's best state as one v_pk_maximum3_f16), alternating; then the aligner and task parity suites
# on the new default build.
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/r3c39
mkdir -p $O
cd $GRAFT_REPO_ROOT
for r in 1 2 3; do
  for L in head ""; do
    N=${L:-max3}
    TAXI2_LIB=libtaxi2_mi355x${L:+_$L}.so timeout -k 10 150 python -u bench.py --steps 8 --warmup 2 --no-cpu-baseline > $O/${N}_$r.json 2> $O/${N}_$r.err || exit $?
  done
done
timeout -k 10 900 python -u -m pytest tests/test_gpu_alignt.py tests/test_gpu_regress.py tests/test_gpu_band.py tests/test_gpu_parity.py tests/test_gpu_walk_strings.py tests/test_gpu_tasks.py -x -q --timeout 300 --timeout-method thread > $O/tests_max3.log 2>&1
