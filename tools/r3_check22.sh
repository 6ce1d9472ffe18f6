# Round 3: the pipelined one-fill aligned_pairs path with the aligner leaving 0 / 16 / 32 CUs to
# the previous block's post-processing (parity first, then the task bench at N = 5 000 each).
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/r3c22
mkdir -p $O
cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest tests/test_gpu_walk_strings.py -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || exit $?
for r in 0 16; do
  TAXI2_PAIRS_RESERVE=$r timeout -k 10 300 python -u tools/bench_task.py --n 5000 > $O/task_reserve$r.json 2> $O/task_reserve$r.err || exit $?
done
