# Trace-band sweep of the packed aligner on one box (bench line + queued-pair count per band)
# usage: BANDS="95 64 48 32 95" bash tools/sweep_band.sh
set -o pipefail
O=gpurun_out/band
mkdir -p $O
i=0
for b in ${BANDS:-95 64 48 32 95}; do
  i=$((i + 1))
  TAXI2_AT_BAND=$b TAXI2_AT_BAND_STATS=1 timeout -k 10 120 python -u bench.py --steps 8 --warmup 2 --no-cpu-baseline > $O/r${i}_b$b.json 2> $O/r${i}_b$b.err || exit $?
done
