# A/B of the candidate build (libtaxi2_mi355x_v3.so) vs the shipped one, its parity suites, and the
# poisoning guard build of the same source on the packed-aligner suites
set -o pipefail
O=gpurun_out/abv3
mkdir -p $O
PYT="python -u -m pytest -x -q --timeout 300 --timeout-method thread"
for r in 1 2; do
  timeout -k 10 120 python -u bench.py --steps 8 --warmup 2 --no-cpu-baseline > $O/a_$r.json 2> $O/a_$r.err || exit $?
  TAXI2_LIB=libtaxi2_mi355x_v3.so timeout -k 10 120 python -u bench.py --steps 8 --warmup 2 --no-cpu-baseline > $O/b_$r.json 2> $O/b_$r.err || exit $?
done
TAXI2_LIB=libtaxi2_mi355x_v3.so timeout -k 10 600 $PYT tests/test_gpu_alignt.py tests/test_gpu_regress.py tests/test_gpu_band.py tests/test_gpu_parity.py tests/test_gpu_tasks.py > $O/tests_v3.log 2>&1 &&
TAXI2_LIB=libtaxi2_mi355x_guard.so timeout -k 10 600 $PYT tests/test_gpu_alignt.py tests/test_gpu_regress.py tests/test_gpu_band.py > $O/tests_guard.log 2>&1
