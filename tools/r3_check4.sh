# Round 3, fourth GPU check: occupancy / out-of-band-skip A/B of the packed aligner (six builds of
# the same source: A2_OCC 6 / 5 / 4 x A2_SKIP_OUT_OF_BAND 1 / 0), the subset-aggregation scaling
# bench (N = 50 000; 2 / 1 000 / 10 000 groups), and a kernel trace of the config-5 task path at
# N = 50 000 (where its reduce time goes).
set -o pipefail
O=gpurun_out/r3c4
mkdir -p $O
for lib in libtaxi2_mi355x.so libtaxi2_mi355x_noskip.so libtaxi2_mi355x_occ4.so libtaxi2_mi355x_occ5.so libtaxi2_mi355x_noskip_occ4.so libtaxi2_mi355x_noskip_occ5.so; do
  TAXI2_LIB=$lib timeout -k 10 150 python -u bench.py --steps 8 --warmup 2 --no-cpu-baseline > $O/ab_$lib.json 2> $O/ab_$lib.err || exit $?
done
timeout -k 10 300 python -u tools/bench_subsets.py --n 50000 > $O/bench_subsets.json 2> $O/bench_subsets.err || exit $?
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_c5 -o c5 -- python3 -u tools/bench_config5_task.py --n 50000 > $O/c5_50k.json 2> $O/c5_50k.err
