# decode launch time with the Kaldi epsilon-queue replay skipped (development timing)
mkdir -p gpurun_out
for D in 0 8; do
VOSK_AMD_DEC_DEBUG=$D timeout -k 10 300 python -u bench.py --workload engine --steps 20 --no-pipeline > gpurun_out/ph2_$D.json 2> gpurun_out/ph2_$D.err || exit $?
python3 -c "import json; d=json.load(open('gpurun_out/ph2_$D.json')); print('debug $D', d['value'], d['roofline']['avg_launch_ms'])"
done
