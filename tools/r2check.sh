# Round-2 HEAD check on the GPU box: skip/noskip A/B bench, gpu suite, smoke, default bench line
# (each step time-limited, && chained)
set -o pipefail
O=gpurun_out/r2c
mkdir -p $O
for r in 1 2; do
  timeout -k 10 120 python -u bench.py --steps 8 --warmup 2 --no-cpu-baseline > $O/skip_$r.json 2> $O/skip_$r.err || exit $?
  TAXI2_LIB=libtaxi2_mi355x_noskip.so timeout -k 10 120 python -u bench.py --steps 8 --warmup 2 --no-cpu-baseline > $O/noskip_$r.json 2> $O/noskip_$r.err || exit $?
done
timeout -k 10 800 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu.log 2>&1 &&
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 &&
timeout -k 10 300 python -u bench.py > $O/bench.json 2> $O/bench.err
