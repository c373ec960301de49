# Round-3 quick check (gpurun helper): selected GPU tests, then the driver's
# bench invocation.   usage: bash tools/r03_quick.sh <tag> [pytest targets...]
TAG=${1:-q}; shift
mkdir -p gpurun_out
export TMPDIR=${TMPDIR:-/tmp}
if [ $# -gt 0 ]; then
  timeout -k 10 600 python -u -m pytest "$@" -x -v --timeout 300 --timeout-method thread > gpurun_out/q_tests_$TAG.log 2>&1
  rc=$?; tail -15 gpurun_out/q_tests_$TAG.log
  [ $rc -ne 0 ] && exit $rc
fi
timeout -k 10 600 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/q_bench_$TAG.json 2> gpurun_out/q_bench_$TAG.err
rc=$?
tail -c 3000 gpurun_out/q_bench_$TAG.json
exit $rc
