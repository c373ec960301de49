# Kaldi-order decoder checks (gpurun helper): usage bash tools/r03_kaldi.sh <tag> <pytest targets...>
TAG=${1:-k}; shift
mkdir -p gpurun_out
export TMPDIR=${TMPDIR:-/tmp}
timeout -k 10 900 python -u -m pytest "$@" -x -v --timeout 300 --timeout-method thread > gpurun_out/k_tests_$TAG.log 2>&1
rc=$?
tail -30 gpurun_out/k_tests_$TAG.log
exit $rc
