set -o pipefail
mkdir -p gpurun_out
export TMPDIR=${TMPDIR:-/tmp}
timeout -k 10 400 python -u -m pytest tests/test_batching.py -x -v --timeout 300 --timeout-method thread > gpurun_out/q_tests_lanes.log 2>&1; rc=$?
tail -12 gpurun_out/q_tests_lanes.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 600 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-single-stream --no-engine-line --lanes 0,0 --streams 128 > gpurun_out/q_bench_lanes.json 2> gpurun_out/q_bench_lanes.err
rc=$?; head -c 1200 gpurun_out/q_bench_lanes.json; exit $rc
