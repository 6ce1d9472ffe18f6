# Same-box A/B of the packed aligner's out-of-band trace skip (libtaxi2_mi355x.so) against the
# always-encode build (libtaxi2_mi355x_noskip.so), then the aligner / long-pair parity tests.
set -o pipefail
O=gpurun_out/ab
mkdir -p $O
for r in 1 2; do
  timeout -k 10 120 python -u bench.py --steps 8 --warmup 2 --no-cpu-baseline > $O/skip_$r.json 2> $O/skip_$r.err || exit $?
  TAXI2_LIB=libtaxi2_mi355x_noskip.so timeout -k 10 120 python -u bench.py --steps 8 --warmup 2 --no-cpu-baseline > $O/noskip_$r.json 2> $O/noskip_$r.err || exit $?
done
timeout -k 10 600 python -u -m pytest tests/test_gpu_alignt.py tests/test_gpu_regress.py tests/test_gpu_long.py tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1
