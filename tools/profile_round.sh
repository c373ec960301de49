# Round profile (gpurun helper): kernel-trace stats of the bench's headline
# leg alone (no secondary legs, so every decode_kernel launch in the trace is
# the headline's), then separate FETCH_SIZE / WRITE_SIZE counter passes of
# the same command (they cannot share a pass on gfx950), summarised by
# tools/pmc_summary.py.
#   usage: bash tools/profile_round.sh <tag> [bench args, default: the driver's --steps 20 --warmup 5]
set -e
TAG=${1:-r01}; shift
BARGS=${@:---steps 20 --warmup 5}
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/prof_$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
ARGS="--no-cpu-baseline --no-single-stream --no-order-line --no-engine-line $BARGS"
echo "bench args: $ARGS" > $OUT/args.txt
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $OUT/trace -o run --output-format csv -- python3 $R/bench.py $ARGS > $OUT/bench_trace.json 2> $OUT/trace.err
timeout -k 10 600 rocprofv3 --pmc FETCH_SIZE -d $OUT/fetch -o run --output-format csv -- python3 $R/bench.py $ARGS > $OUT/bench_fetch.json 2> $OUT/fetch.err
timeout -k 10 600 rocprofv3 --pmc WRITE_SIZE -d $OUT/write -o run --output-format csv -- python3 $R/bench.py $ARGS > $OUT/bench_write.json 2> $OUT/write.err
python3 $R/tools/pmc_summary.py $OUT > $OUT/pmc_summary.json
cat $OUT/pmc_summary.json
