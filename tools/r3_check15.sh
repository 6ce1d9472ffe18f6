# Round 3: (1) long shapes (1 200 / 1 500 / 2 000 bp: the 4-fill-wave packed variants) on the
# always-encode default, the skip build and the round-2 build, alternated; (2) the (4, 4) packed
# shape (four fill waves of 4 columns per walker) at 1 000 bp: aligner parity on its build, then an
# A/B against the default (8, 2).
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/r3c15
mkdir -p $O
cd $GRAFT_REPO_ROOT
for r in 1 2; do
  for lib in libtaxi2_mi355x.so libtaxi2_mi355x_skip.so libtaxi2_mi355x_r2.so; do
    TAXI2_LIB=$lib timeout -k 10 300 python -u tools/bench_long.py > $O/long_${lib}_$r.json 2> $O/long_${lib}_$r.err || exit $?
  done
done
TAXI2_LIB=libtaxi2_mi355x_k4w4.so timeout -k 10 600 python -u -m pytest tests/test_gpu_alignt.py tests/test_gpu_band.py -x -q --timeout 300 --timeout-method thread > $O/tests_k4w4.log 2>&1 || exit $?
for r in 1 2; do
  for lib in libtaxi2_mi355x.so libtaxi2_mi355x_k4w4.so; do
    TAXI2_LIB=$lib timeout -k 10 150 python -u bench.py --steps 8 --warmup 2 --no-cpu-baseline > $O/ab_${lib}_$r.json 2> $O/ab_${lib}_$r.err || exit $?
  done
done
