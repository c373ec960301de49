# Kaldi-order decoder tests, then the Kaldi-order phase counters (gpurun helper)
TAG=${1:-k}
mkdir -p gpurun_out
export TMPDIR=${TMPDIR:-/tmp}
timeout -k 10 600 python -u -m pytest tests/test_kaldi_order_gpu.py tests/test_eps_frames_gpu.py tests/test_api_gpu.py tests/test_recognizer_endpoint_gpu.py tests/test_lookahead_gpu.py -x -v --timeout 300 --timeout-method thread > gpurun_out/kq_$TAG.log 2>&1
rc=$?; tail -8 gpurun_out/kq_$TAG.log
[ $rc -ne 0 ] && exit $rc
VOSK_AMD_DEC_PROFILE=1 timeout -k 10 300 python -u bench.py --workload engine --order kaldi --steps 20 --no-pipeline > gpurun_out/phases_kaldi_$TAG.json 2> gpurun_out/phases_kaldi_$TAG.err || exit $?
python3 -c "import json; d=json.load(open('gpurun_out/phases_kaldi_$TAG.json')); print('kaldi', d['value'], d['roofline']['avg_launch_ms'], json.dumps(d.get('decoder_phase_clocks_per_frame')))"
