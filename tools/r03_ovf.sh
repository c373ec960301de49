# overflow test first (it faulted), then the full GPU suite and the driver bench
TAG=${1:-o}
mkdir -p gpurun_out
export TMPDIR=${TMPDIR:-/tmp}
timeout -k 10 300 python -u -m pytest tests/test_decoder_overflow_gpu.py -x -v --timeout 120 --timeout-method thread > gpurun_out/ovf_$TAG.log 2>&1
rc=$?; tail -5 gpurun_out/ovf_$TAG.log
[ $rc -ne 0 ] && exit $rc
bash tools/r03_suite.sh $TAG
