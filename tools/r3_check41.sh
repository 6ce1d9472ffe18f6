# Round 3: the value-range extremes of the maximum3 fill (new test) and the packed aligner suite.
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/r3c41
mkdir -p $O
cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest tests/test_gpu_alignt.py -x -v --timeout 300 --timeout-method thread > $O/tests_alignt.log 2>&1
