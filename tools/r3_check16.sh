# Round 3: 4-fill-wave shapes back on the sign-digit trace (parity suites for the packed aligner,
# long-pair bench), and config 4 on a 65 536-query slice (6.6e8 pairs: a 15x smaller extrapolation
# to the 1e6 x 1e4 job than the 1 024-query slice).
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/r3c16
mkdir -p $O
cd $GRAFT_REPO_ROOT
timeout -k 10 900 python -u -m pytest tests/test_gpu_alignt.py tests/test_gpu_band.py tests/test_gpu_long.py tests/test_gpu_walk_strings.py tests/test_gpu_regress.py tests/test_gpu_parity.py -x -v --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || exit $?
timeout -k 10 300 python -u tools/bench_long.py > $O/long.json 2> $O/long.err || exit $?
timeout -k 10 600 python -u tools/bench_configs.py --config4 --q-slice 65536 --steps 1 > $O/config4_65536.json 2> $O/config4.err
