# full GPU suite (incl. the scale tests), then the driver's bench line (gpurun helper)
TAG=${1:-f}
mkdir -p gpurun_out
export TMPDIR=${TMPDIR:-/tmp}
timeout -k 10 1100 python -u -m pytest tests -m gpu -x -v --timeout 600 --timeout-method thread --durations=20 > gpurun_out/suite_$TAG.log 2>&1
rc=$?
tail -30 gpurun_out/suite_$TAG.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 500 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/suite_bench_$TAG.json 2> gpurun_out/suite_bench_$TAG.err
rc=$?
head -c 1200 gpurun_out/suite_bench_$TAG.json
exit $rc
