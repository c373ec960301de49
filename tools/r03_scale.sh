# decoder phase clocks (both orders), then the 256-stream scale tests (gpurun helper)
mkdir -p gpurun_out
export TMPDIR=${TMPDIR:-/tmp}
bash tools/r03_phases.sh || exit $?
timeout -k 10 900 python -u -m pytest tests/test_scale_gpu.py -x -v --timeout 600 --timeout-method thread --durations=5 > gpurun_out/scale_${1:-a}.log 2>&1
rc=$?; tail -15 gpurun_out/scale_${1:-a}.log; exit $rc
