# Kaldi-order decoder tests first, then the full suite, phases and bench (gpurun helper)
TAG=${1:-k}
mkdir -p gpurun_out
export TMPDIR=${TMPDIR:-/tmp}
timeout -k 10 600 python -u -m pytest tests/test_kaldi_order_gpu.py tests/test_eps_frames_gpu.py tests/test_xvector_gpu.py tests/test_spk_concurrent_gpu.py tests/test_api_gpu.py -x -v --timeout 300 --timeout-method thread > gpurun_out/kq_$TAG.log 2>&1
rc=$?; tail -8 gpurun_out/kq_$TAG.log
[ $rc -ne 0 ] && exit $rc
bash tools/r03_full3.sh $TAG
