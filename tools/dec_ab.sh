# decoder phase probe with and without lattice links, in order (gpurun helper)
set -e
mkdir -p gpurun_out
for mode in "--no-lattice" ""; do
  VOSK_AMD_DEC_PROFILE=1 timeout -k 10 300 python bench.py --steps 20 --warmup 4 --no-cpu-baseline --no-pipeline $mode > gpurun_out/probe.json
  python - "$mode" <<'PY'
import json,sys
d=json.loads(open("gpurun_out/probe.json").read().strip().splitlines()[-1])
print(sys.argv[1] or "lattice", d["value"], d["ms_per_step"], d.get("stages_ms_per_step"), d["decoder"])
print("  phases/frame", d.get("decoder_phase_clocks_per_frame"))
PY
done
