# lattice parity + decoder regression + bench with / without lattice links (gpurun helper)
set -e
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_lattice_gpu.py tests/test_gpu_parity.py tests/test_silence_weighting_gpu.py -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/lat_tests.log 2>&1
for mode in "--no-lattice" ""; do
  timeout -k 10 300 python bench.py --steps 20 --warmup 4 --no-cpu-baseline $mode > gpurun_out/lat_bench.json
  python - "$mode" <<'PY'
import json,sys
d=json.loads(open("gpurun_out/lat_bench.json").read().strip().splitlines()[-1])
print(sys.argv[1] or "lattice", d["value"], d["ms_per_step"], d.get("stages_ms_per_step"))
PY
done
