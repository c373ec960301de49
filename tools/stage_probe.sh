# Per-stage GPU timing + decoder phase clocks at 1 and 256 streams (gpurun helper).
set -e
mkdir -p gpurun_out
export VOSK_AMD_DEC_PROFILE=1
timeout -k 10 300 python -m pytest tests/test_gpu_parity.py -x -q 2>&1 | tail -3
for s in 1 256; do
timeout -k 10 300 python bench.py --streams $s --steps 20 --warmup 4 --no-cpu-baseline > gpurun_out/probe_$s.json
python - $s <<'PY'
import json,sys
d=json.loads(open(f"gpurun_out/probe_{sys.argv[1]}.json").read().strip().splitlines()[-1])
print(sys.argv[1], d["value"], d.get("stages_ms_per_step"), d.get("decoder_phase_clocks_per_frame"))
PY
done
