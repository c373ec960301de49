# 1024-thread decoder variant: parity, in-order decoder A/B, pipelined bench (gpurun helper)
set -e
mkdir -p gpurun_out
cp vosk-api_amd/vosk_dt/libvosk.so vosk-api_amd/vosk/libvosk.so
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_lattice_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/dt_tests.log 2>&1
bash tools/dec_ab.sh
timeout -k 10 300 python bench.py --steps 30 --warmup 6 --no-cpu-baseline > gpurun_out/dt_bench.json
python -c "
import json; d=json.loads(open('gpurun_out/dt_bench.json').read().strip().splitlines()[-1]); print('pipeline', d['value'], d['ms_per_step'], d['stages_ms_per_step'])"
