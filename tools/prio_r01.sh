# stream-priority experiment on the pipelined bench (gpurun helper)
set -e
mkdir -p gpurun_out
for m in 0 1 2; do
  VOSK_AMD_STREAM_PRIO=$m timeout -k 10 300 python bench.py --steps 30 --warmup 6 --no-cpu-baseline > gpurun_out/prio.json
  python - $m <<'PY'
import json,sys
d=json.loads(open("gpurun_out/prio.json").read().strip().splitlines()[-1])
print("prio", sys.argv[1], d["value"], d["ms_per_step"], d.get("stages_ms_per_step"))
PY
done
