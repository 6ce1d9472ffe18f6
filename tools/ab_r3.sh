# Same-box A/B of two engine builds (bench line, alternating), then the aligner parity suites on B.
# usage: bash tools/ab_r3.sh LIB_A LIB_B [OUTDIR]   (file names under taxi2_amd/_lib)
set -o pipefail
O=${3:-gpurun_out/ab3}
mkdir -p $O
for r in 1 2; do
  TAXI2_LIB=$1 timeout -k 10 150 python -u bench.py --steps 8 --warmup 2 --no-cpu-baseline > $O/a_$r.json 2> $O/a_$r.err || exit $?
  TAXI2_LIB=$2 TAXI2_AT_BAND_STATS=1 timeout -k 10 150 python -u bench.py --steps 8 --warmup 2 --no-cpu-baseline > $O/b_$r.json 2> $O/b_$r.err || exit $?
done
TAXI2_LIB=$2 timeout -k 10 900 python -u -m pytest tests/test_gpu_alignt.py tests/test_gpu_regress.py tests/test_gpu_band.py tests/test_gpu_parity.py -x -v --timeout 300 --timeout-method thread > $O/tests_b.log 2>&1
