# Round 3: config-3 throughput under other scores (generic Gotoh, linear) beside the default.
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/r3c18
mkdir -p $O
cd $GRAFT_REPO_ROOT
timeout -k 10 400 python -u tools/bench_scores.py > $O/bench_scores.json 2> $O/bench_scores.err
