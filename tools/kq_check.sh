# Kaldi-order decoder parity tests, then the phase profile of both orders (gpurun helper)
# usage: bash tools/kq_check.sh <tag> [extra pytest files]
TAG=${1:-k}; shift
mkdir -p gpurun_out
export TMPDIR=${TMPDIR:-/tmp}
timeout -k 10 600 python -u -m pytest tests/test_kaldi_order_gpu.py tests/test_eps_frames_gpu.py "$@" -x -q \
    --timeout 300 --timeout-method thread > gpurun_out/kq_$TAG.log 2>&1
rc=$?; tail -5 gpurun_out/kq_$TAG.log
[ $rc -ne 0 ] && exit $rc
bash tools/phases.sh $TAG
