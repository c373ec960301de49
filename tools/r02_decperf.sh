# Decoder change check (gpurun helper): decoder parity tests, then the
# engine-only bench with phase clocks and a short public-API bench on the
# lookahead small-en-us-scale model.  usage: bash tools/r02_decperf.sh <tag> [notests]
set -e
TAG=${1:-x}
mkdir -p gpurun_out
export TMPDIR=${TMPDIR:-/tmp}
if [ "$2" != notests ]; then
  timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_decoder_prune_gpu.py tests/test_lattice_gpu.py \
    tests/test_large_graph_gpu.py -x -v --timeout 300 --timeout-method thread > gpurun_out/decperf_tests_$TAG.log 2>&1 \
    || { grep -E "PASS|FAIL|Error|assert" gpurun_out/decperf_tests_$TAG.log | tail -30; exit 1; }
  tail -2 gpurun_out/decperf_tests_$TAG.log
fi
VOSK_AMD_DEC_PROFILE=1 timeout -k 10 600 python bench.py --workload engine --steps 20 --no-cpu-baseline \
  --no-single-stream > gpurun_out/decperf_eng_$TAG.json 2> gpurun_out/decperf_eng_$TAG.err
python -c "
import json; d=json.load(open('gpurun_out/decperf_eng_$TAG.json'))
print('engine', d['value'], d['stages_ms_per_step'], d['decoder'])
print({k: v for k, v in d.get('decoder_phase_clocks_per_frame', {}).items()})"
timeout -k 10 600 python bench.py --stream-seconds 20 --no-cpu-baseline --no-single-stream --no-engine-line \
  > gpurun_out/decperf_api_$TAG.json 2> gpurun_out/decperf_api_$TAG.err
python -c "
import json; d=json.load(open('gpurun_out/decperf_api_$TAG.json'))
print('api', d['value'], d['ms_per_step'], d['p50_chunk_latency_ms'], d['finish_ms'], d['gpu_ms_per_step'], d['roofline']['avg_launch_ms'])"
