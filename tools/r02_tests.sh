# Selected GPU tests (gpurun helper): usage bash tools/r02_tests.sh <tag> <pytest args...>
TAG=${1:-x}; shift
mkdir -p gpurun_out
export TMPDIR=${TMPDIR:-/tmp}
timeout -k 10 900 python -u -m pytest "$@" -x -v --timeout 300 --timeout-method thread \
  -o faulthandler_timeout=280 > gpurun_out/tests_$TAG.log 2>&1
rc=$?
grep -E "PASS|FAIL|ERROR|Error|assert|passed|failed" gpurun_out/tests_$TAG.log | tail -40
exit $rc
