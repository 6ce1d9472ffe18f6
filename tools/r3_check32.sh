# Round 3: single-exit hop loops in both walkers (the branch-free walker had two copies of the walk
# state and a scratch reload per hop) -- aligner suites, long-shape bench (W = 4 shapes use the
# branchy walker), then a same-box A/B against the previous build (bf).
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/r3c32
mkdir -p $O
cd $GRAFT_REPO_ROOT
timeout -k 10 700 python -u -m pytest tests/test_gpu_alignt.py tests/test_gpu_band.py tests/test_gpu_regress.py tests/test_gpu_parity.py tests/test_gpu_walk_strings.py tests/test_gpu_long.py -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || exit $?
for r in 1 2 3; do
  TAXI2_LIB=libtaxi2_mi355x_bf.so timeout -k 10 120 python -u bench.py --steps 8 --warmup 2 --no-cpu-baseline > $O/bf_$r.json 2> $O/bf_$r.err || exit $?
  timeout -k 10 120 python -u bench.py --steps 8 --warmup 2 --no-cpu-baseline > $O/se_$r.json 2> $O/se_$r.err || exit $?
done
