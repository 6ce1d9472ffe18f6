# Round 3, twelfth GPU check: A/B of packed-aligner experiments on one box (timing only):
# the per-column gap-open constants from a uniform register instead of LDS (upper bound of removing
# those reads; inexact at the end-gap column), and the fill waves at a higher issue priority.
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/r3c12
mkdir -p $O
cd $GRAFT_REPO_ROOT
for r in 1 2; do
  for lib in libtaxi2_mi355x.so libtaxi2_mi355x_exp_nocolc.so libtaxi2_mi355x_exp_prio1.so libtaxi2_mi355x_exp_prio3.so; do
    TAXI2_LIB=$lib timeout -k 10 150 python -u bench.py --steps 8 --warmup 2 --no-cpu-baseline > $O/ab_${lib}_$r.json 2> $O/ab_${lib}_$r.err || exit $?
  done
done
