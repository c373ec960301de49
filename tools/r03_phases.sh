# Decoder phase clocks of the engine bench in both orders (gpurun helper)
mkdir -p gpurun_out
export TMPDIR=${TMPDIR:-/tmp}
for ORD in kaldi parallel; do
  VOSK_AMD_DEC_ORDER=$ORD VOSK_AMD_DEC_PROFILE=1 timeout -k 10 300 python -u bench.py --workload engine --steps 20 --no-pipeline > gpurun_out/phases_$ORD.json 2> gpurun_out/phases_$ORD.err || exit $?
  python3 -c "import json; d=json.load(open('gpurun_out/phases_$ORD.json')); print('$ORD', d['value'], d['roofline']['avg_launch_ms'], json.dumps(d.get('decoder_phase_clocks_per_frame')))"
done
