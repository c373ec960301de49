# one GPU test file / node id with a heartbeat (gpurun helper): r03_one.sh TAG TEST [TEST...]
TAG=$1; shift
mkdir -p gpurun_out
export TMPDIR=${TMPDIR:-/tmp}
(while true; do sleep 50; echo "[hb] $(date +%T)" >> gpurun_out/hb_$TAG.log; done) &
HB=$!
trap "kill $HB" EXIT
timeout -k 10 400 python -u -m pytest "$@" -x -v -s --timeout 300 --timeout-method thread > gpurun_out/one_$TAG.log 2>&1
rc=$?; tail -5 gpurun_out/one_$TAG.log
exit $rc
