# GPU test suite (gpurun helper): usage bash tools/gpu_tests.sh <tag> [pytest args]
TAG=${1:-run}; shift
mkdir -p gpurun_out
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread "$@" > gpurun_out/gpu_tests_$TAG.log 2>&1
rc=$?
tail -25 gpurun_out/gpu_tests_$TAG.log
exit $rc
