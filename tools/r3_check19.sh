# Round 3: generic-score packed kernels at 4 waves per SIMD (128 VGPRs) vs the build that asks
# for 6 and ends at 3 (144 VGPRs): aligner parity on the 4-wave build, then the scores bench on both.
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/r3c19
mkdir -p $O
cd $GRAFT_REPO_ROOT
TAXI2_LIB=libtaxi2_mi355x_gen4.so timeout -k 10 600 python -u -m pytest tests/test_gpu_alignt.py tests/test_gpu_band.py -x -q --timeout 300 --timeout-method thread > $O/tests_gen4.log 2>&1 || exit $?
for r in 1 2; do
  for lib in libtaxi2_mi355x.so libtaxi2_mi355x_gen4.so; do
    TAXI2_LIB=$lib timeout -k 10 300 python -u tools/bench_scores.py > $O/scores_${lib}_$r.json 2> $O/scores_${lib}_$r.err || exit $?
  done
done
