set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r1end_gpu.log 2>&1 || exit $?
timeout -k 10 200 python -u tools/bench_ragged.py --lo 2100 --hi 2600 --nseq 1500 --batch 32768 --reps 2 > gpurun_out/r1end_ragged.log 2>&1 || exit $?
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r1end_smoke.log 2>&1 || exit $?
timeout -k 10 300 python -u bench.py > gpurun_out/r1end_bench.log 2>&1 || exit $?
