# Round 3: task-level A/B of the aligned_pairs path at N = 5 000 -- the sequential one-fill form
# (TAXI2_PAIRS_SEQ=1), the two-stream pipeline with no CU reserve, and with 16 CUs reserved.
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/r3c25
mkdir -p $O
cd $GRAFT_REPO_ROOT
for r in 1 2; do
  TAXI2_PAIRS_SEQ=1 timeout -k 10 200 python -u tools/bench_task.py --n 5000 > $O/seq_$r.json 2> $O/seq_$r.err || exit $?
  TAXI2_PAIRS_RESERVE=0 timeout -k 10 200 python -u tools/bench_task.py --n 5000 > $O/pipe0_$r.json 2> $O/pipe0_$r.err || exit $?
  TAXI2_PAIRS_RESERVE=16 timeout -k 10 200 python -u tools/bench_task.py --n 5000 > $O/pipe16_$r.json 2> $O/pipe16_$r.err || exit $?
done
