# API bench: the driver's invocation, then the 60-s workload (gpurun helper)
# usage: bash tools/api_bench.sh <tag>
TAG=${1:-api}
mkdir -p gpurun_out
export TMPDIR=${TMPDIR:-/tmp}
VOSK_AMD_STEP_PROFILE=1 timeout -k 10 600 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline \
    > gpurun_out/api_${TAG}_6s.json 2> gpurun_out/api_${TAG}_6s.err || exit $?
python3 -c "import json; d=json.load(open('gpurun_out/api_${TAG}_6s.json')); print('6s', d['value'], d['decoder_order'], d['finish_ms'], d['gpu_ms_per_step'], {k: (d[k]['value'], d[k]['finish_ms']) for k in ('kaldi_order','order_independent') if k in d})"
timeout -k 10 900 python -u bench.py --no-cpu-baseline --no-single-stream --no-engine-line --no-order-line \
    > gpurun_out/api_${TAG}_60s.json 2> gpurun_out/api_${TAG}_60s.err || exit $?
python3 -c "import json; d=json.load(open('gpurun_out/api_${TAG}_60s.json')); print('60s', d['value'], d['decoder_order'], d['finish_ms'], d['gpu_ms_per_step'], d['result_production'])"
