mkdir -p gpurun_out
VOSK_AMD_DEC_PROFILE=1 timeout -k 10 300 python -u bench.py --workload engine --steps 20 --no-pipeline > gpurun_out/phases_diag.json 2> gpurun_out/phases_diag.err || exit $?
python3 -c "import json; d=json.load(open('gpurun_out/phases_diag.json')); print(d['value'], d['roofline']['avg_launch_ms'], json.dumps(d.get('decoder_phase_clocks_per_frame')))"
