# full GPU suite, decoder phase clocks in both orders, the driver's bench line (gpurun helper)
TAG=${1:-f}
mkdir -p gpurun_out
export TMPDIR=${TMPDIR:-/tmp}
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 600 --timeout-method thread --durations=20 > gpurun_out/suite_$TAG.log 2>&1
rc=$?
tail -25 gpurun_out/suite_$TAG.log
[ $rc -ne 0 ] && exit $rc
for ORD in parallel kaldi; do
  VOSK_AMD_DEC_PROFILE=1 timeout -k 10 300 python -u bench.py --workload engine --order $ORD --steps 20 --no-pipeline > gpurun_out/phases_${ORD}_$TAG.json 2> gpurun_out/phases_${ORD}_$TAG.err || exit $?
  python3 -c "import json; d=json.load(open('gpurun_out/phases_${ORD}_$TAG.json')); print('$ORD', d['value'], d['roofline']['avg_launch_ms'], json.dumps(d['decoder']), json.dumps(d.get('decoder_phase_clocks_per_frame')))"
done
timeout -k 10 500 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/suite_bench_$TAG.json 2> gpurun_out/suite_bench_$TAG.err
rc=$?
head -c 600 gpurun_out/suite_bench_$TAG.json
exit $rc
