# Trace-band sweep of the packed aligner on one box (bench line + queued-pair count per band)
set -o pipefail
O=gpurun_out/band
mkdir -p $O
for b in 95 64 48 32 95; do
  TAXI2_AT_BAND=$b TAXI2_AT_BAND_STATS=1 timeout -k 10 120 python -u bench.py --steps 8 --warmup 2 --no-cpu-baseline > $O/b$b.json 2> $O/b$b.err || exit $?
done
