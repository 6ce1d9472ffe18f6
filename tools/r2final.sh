# Round-2 HEAD evidence on one box: profile (valu_peak, bench, rocprofv3 stats, PMC passes), then the
# GPU suite, smoke and the default bench line.  Each GPU step time-limited, && chained.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
PROF_NAME=prof_r2c bash $R/tools/profile_r2.sh > $R/gpurun_out/prof_r2c.log 2>&1 &&
cd $R && mkdir -p gpurun_out/r2f &&
timeout -k 10 800 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r2f/gpu.log 2>&1 &&
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r2f/smoke.log 2>&1 &&
timeout -k 10 300 python -u bench.py > gpurun_out/r2f/bench.json 2> gpurun_out/r2f/bench.err &&
timeout -k 10 400 python -u tools/bench_configs.py --config5 > gpurun_out/r2f/config5.json 2> gpurun_out/r2f/config5.err
