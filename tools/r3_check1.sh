# Round 3, first GPU check: A/B of the raw-difference packed aligner (bench, alternating with the
# round-2 build), the aligner + pre-aligned parity suites on the new build, then configs 2 / 5 with
# the tiled pre-aligned kernel.
set -o pipefail
O=gpurun_out/r3c1
mkdir -p $O
bash tools/ab_r3.sh libtaxi2_mi355x_r2.so libtaxi2_mi355x.so $O || exit $?
timeout -k 10 300 python -u tools/bench_configs.py --config2 --config5 > $O/configs.json 2> $O/configs.err || exit $?
TAXI2_PRE_NOTILE=1 timeout -k 10 300 python -u tools/bench_configs.py --config2 > $O/configs_notile.json 2> $O/configs_notile.err
