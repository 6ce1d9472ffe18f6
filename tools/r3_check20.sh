# Round 3: the pipelined one-fill aligned_pairs path (alignment of block b on one stream, the
# previous block's compaction / metrics / text / D2H / write on another; text kernels fully on the
# device) -- task parity suites, then the task bench.
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/r3c20
mkdir -p $O
cd $GRAFT_REPO_ROOT
timeout -k 10 700 python -u -m pytest tests/test_gpu_walk_strings.py tests/test_gpu_tasks.py tests/test_gpu_alignt.py -x -v --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || exit $?
timeout -k 10 700 python -u tools/bench_task.py > $O/bench_task.json 2> $O/bench_task.err
