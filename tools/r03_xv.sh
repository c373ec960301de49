# batched x-vector tests, Kaldi-order decoder tests, Kaldi phase counters, config-5 speaker bench (gpurun helper)
TAG=${1:-x}
mkdir -p gpurun_out
export TMPDIR=${TMPDIR:-/tmp}
timeout -k 10 600 python -u -m pytest tests/test_xvector_gpu.py tests/test_spk_concurrent_gpu.py tests/test_kaldi_order_gpu.py -x -v --timeout 300 --timeout-method thread > gpurun_out/xv_$TAG.log 2>&1
rc=$?; tail -8 gpurun_out/xv_$TAG.log
[ $rc -ne 0 ] && exit $rc
VOSK_AMD_DEC_PROFILE=1 timeout -k 10 300 python -u bench.py --workload engine --order kaldi --steps 20 --no-pipeline > gpurun_out/phases_kaldi_$TAG.json 2> gpurun_out/phases_kaldi_$TAG.err || exit $?
python3 -c "import json; d=json.load(open('gpurun_out/phases_kaldi_$TAG.json')); print('kaldi', d['value'], d['roofline']['avg_launch_ms'], json.dumps(d.get('decoder_phase_clocks_per_frame')))"
timeout -k 10 400 python -u bench.py --workload spk --steps 10 --warmup 2 > gpurun_out/spk_bench_$TAG.json 2> gpurun_out/spk_bench_$TAG.err
rc=$?
head -c 1500 gpurun_out/spk_bench_$TAG.json
exit $rc
