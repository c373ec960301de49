# Stage times in order (isolated kernels) and pipelined, with decoder phase
# clocks (gpurun helper).
set -e
mkdir -p gpurun_out
for mode in "--no-pipeline" ""; do
  VOSK_AMD_DEC_PROFILE=1 timeout -k 10 300 python bench.py --steps 20 --warmup 4 --no-cpu-baseline $mode > gpurun_out/probe.json
  python - "$mode" <<'PY'
import json,sys
d=json.loads(open("gpurun_out/probe.json").read().strip().splitlines()[-1])
print(sys.argv[1] or "pipeline", d["value"], d["ms_per_step"], d.get("stages_ms_per_step"))
print("  phases/frame", d.get("decoder_phase_clocks_per_frame"))
PY
done
