# Other BASELINE configs and long lengths on the HEAD build (one box)
set -o pipefail
O=gpurun_out/r2cfg
mkdir -p $O
timeout -k 10 300 python -u tools/bench_configs.py --config2 --config4 > $O/configs.json 2> $O/configs.err &&
timeout -k 10 300 python -u tools/bench_long.py > $O/long.json 2> $O/long.err &&
timeout -k 10 200 python -u tools/bench_ncd.py > $O/ncd.json 2> $O/ncd.err
