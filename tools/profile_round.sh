# Round profile (gpurun helper): kernel-trace stats of the default bench
# command, then separate FETCH_SIZE / WRITE_SIZE counter passes (they cannot
# share a pass on gfx950), summarised by tools/pmc_summary.py.
#   usage: bash tools/profile_round.sh <tag>
set -e
TAG=${1:-r01}
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/prof_$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $OUT/trace -o run --output-format csv -- python3 $R/bench.py --no-cpu-baseline --no-single-stream > $OUT/bench_trace.json 2> $OUT/trace.err
timeout -k 10 600 rocprofv3 --pmc FETCH_SIZE -d $OUT/fetch -o run --output-format csv -- python3 $R/bench.py --no-cpu-baseline --no-single-stream --steps 10 --warmup 2 > $OUT/bench_fetch.json 2> $OUT/fetch.err
timeout -k 10 600 rocprofv3 --pmc WRITE_SIZE -d $OUT/write -o run --output-format csv -- python3 $R/bench.py --no-cpu-baseline --no-single-stream --steps 10 --warmup 2 > $OUT/bench_write.json 2> $OUT/write.err
python3 $R/tools/pmc_summary.py $OUT > $OUT/pmc_summary.json
cat $OUT/pmc_summary.json
