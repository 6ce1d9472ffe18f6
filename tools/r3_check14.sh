# Round 3: the other BASELINE configs, long lengths and NCD on HEAD (one box): config 2 stand-in,
# config 4 slice, config 5 pre-aligned at full size, packed long shapes, raw NCD.
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/r3c14
mkdir -p $O
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u tools/bench_configs.py --config2 --config4 --config5 > $O/configs.json 2> $O/configs.err &&
timeout -k 10 300 python -u tools/bench_long.py > $O/long.json 2> $O/long.err &&
timeout -k 10 200 python -u tools/bench_ncd.py > $O/ncd.json 2> $O/ncd.err
