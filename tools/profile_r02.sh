# Round-2 bench + profile (gpurun helper): the default bench line, then the
# kernel-trace stats of the public-API bench and separate FETCH_SIZE /
# WRITE_SIZE counter passes, summarised by tools/pmc_summary.py.
#   usage: bash tools/profile_r02.sh <tag> [nobench]
set -e
TAG=${1:-r02}
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/prof_$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
if [ "$2" != nobench ]; then
  timeout -k 10 900 python3 $R/bench.py > $OUT/bench.json 2> $OUT/bench.err
  tail -c 1500 $OUT/bench.json
fi
ARGS="--stream-seconds 20 --no-cpu-baseline --no-single-stream --no-engine-line"
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $OUT/trace -o run --output-format csv -- python3 $R/bench.py $ARGS > $OUT/bench_trace.json 2> $OUT/trace.err
echo trace done
timeout -k 10 600 rocprofv3 --pmc FETCH_SIZE -d $OUT/fetch -o run --output-format csv -- python3 $R/bench.py $ARGS > $OUT/bench_fetch.json 2> $OUT/fetch.err
echo fetch done
timeout -k 10 600 rocprofv3 --pmc WRITE_SIZE -d $OUT/write -o run --output-format csv -- python3 $R/bench.py $ARGS > $OUT/bench_write.json 2> $OUT/write.err
python3 $R/tools/pmc_summary.py $OUT > $OUT/pmc_summary.json
python3 -c "import json; d=json.load(open('$OUT/pmc_summary.json')); print('decode hbm bytes/launch', d.get('hbm_bytes_per_launch'))"
