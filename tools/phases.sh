# Decoder launch times and phase clocks of the engine bench in both
# token-passing orders (gpurun helper).  usage: bash tools/phases.sh <tag> [extra bench args]
TAG=${1:-p}; shift
mkdir -p gpurun_out
export TMPDIR=${TMPDIR:-/tmp}
for ord in parallel kaldi; do
  timeout -k 10 300 python -u bench.py --workload engine --order $ord --steps 20 \
      --no-pipeline --no-cpu-baseline "$@" > gpurun_out/launch_${TAG}_$ord.json 2> gpurun_out/launch_${TAG}_$ord.err || exit $?
  python3 -c "import json,sys; d=json.load(open('gpurun_out/launch_${TAG}_$ord.json')); print('$ord (no profile)', d['value'], d['stages_ms_per_step'])"
  VOSK_AMD_DEC_PROFILE=1 timeout -k 10 300 python -u bench.py --workload engine --order $ord --steps 20 \
      --no-pipeline --no-cpu-baseline "$@" > gpurun_out/phases_${TAG}_$ord.json 2> gpurun_out/phases_${TAG}_$ord.err || exit $?
  python3 -c "import json,sys; d=json.load(open('gpurun_out/phases_${TAG}_$ord.json')); print('$ord (profile)', d['value'], d['stages_ms_per_step'], d['decoder'])"
done
