# Round 3: kernel trace of the pipelined aligned_pairs path (does the previous block's text run
# beside the next block's alignment?), N = 3 000, reserve 16 CUs.
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/r3c23
mkdir -p $O
export TMPDIR=/tmp
cd /tmp
TAXI2_PAIRS_RESERVE=16 timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/trace -o run -- \
    python3 $GRAFT_REPO_ROOT/tools/bench_task.py --n 3000 > $O/task.json 2> $O/task.err
