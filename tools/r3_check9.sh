# Round 3, ninth GPU check: the tiled pre-aligned kernel at the config-5 shape under rocprofv3 --
# kernel trace, then FETCH_SIZE and WRITE_SIZE in passes of their own (tools/bench_configs.py
# --config5: 200 000 x 1 000 columns, p / jc / k2p, all 2.0e10 pairs in 2^26-pair launches).
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/r3c9
mkdir -p $O
export TMPDIR=/tmp
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/pre_trace -o run -- \
    python3 $GRAFT_REPO_ROOT/tools/bench_configs.py --config5 > $O/pre_trace.json 2> $O/pre_trace.err &&
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex k_prealigned --output-format csv -d $O/pre_fetch -o run -- \
    python3 $GRAFT_REPO_ROOT/tools/bench_configs.py --config5 > $O/pre_fetch.json 2> $O/pre_fetch.err &&
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex k_prealigned --output-format csv -d $O/pre_write -o run -- \
    python3 $GRAFT_REPO_ROOT/tools/bench_configs.py --config5 > $O/pre_write.json 2> $O/pre_write.err &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/sub_trace -o run -- \
    python3 $GRAFT_REPO_ROOT/tools/bench_subsets.py --n 50000 --groups 2 1000 > $O/sub_trace.json 2> $O/sub_trace.err
