# Debug one batch test with lane tracing (gpurun helper)
mkdir -p gpurun_out
export TMPDIR=${TMPDIR:-/tmp}
VOSK_AMD_BATCH_TRACE=1 timeout -k 10 240 python -u -m pytest "$@" -x -v -s --timeout 200 --timeout-method thread \
  -o faulthandler_timeout=150 > gpurun_out/dbg.log 2>&1
rc=$?
tail -60 gpurun_out/dbg.log
exit $rc
