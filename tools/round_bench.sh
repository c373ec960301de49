# Full default bench (with the CPU baseline) + round profile (gpurun helper).
#   usage: bash tools/round_bench.sh <tag>
set -e
TAG=${1:-r01}
mkdir -p gpurun_out
timeout -k 10 900 python bench.py > gpurun_out/bench_full_$TAG.json 2> gpurun_out/bench_full_$TAG.err
tail -1 gpurun_out/bench_full_$TAG.json
bash tools/profile_round.sh $TAG > /dev/null
python3 -c "import json; d=json.load(open('gpurun_out/prof_$TAG/pmc_summary.json')); print('decode hbm bytes/launch', d.get('hbm_bytes_per_launch'))"
