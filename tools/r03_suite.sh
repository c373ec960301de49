# Full GPU suite + the driver's bench invocation (gpurun helper): bash tools/r03_suite.sh <tag>
TAG=${1:-s}
mkdir -p gpurun_out
export TMPDIR=${TMPDIR:-/tmp}
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread --durations=15 > gpurun_out/suite_$TAG.log 2>&1
rc=$?
tail -40 gpurun_out/suite_$TAG.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 500 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/suite_bench_$TAG.json 2> gpurun_out/suite_bench_$TAG.err
rc=$?
head -c 1500 gpurun_out/suite_bench_$TAG.json
exit $rc
