# Library variants A/B on the engine bench (gpurun helper; development):
# usage: bash tools/exp_variants.sh <variant dirs under build_exp/...>
# "base" = the in-tree build.  Prints decode ms per launch and engine xRT.
set -e
mkdir -p gpurun_out
export TMPDIR=${TMPDIR:-/tmp}
cp vosk-api_amd/vosk/libvosk.so gpurun_out/libvosk_base.so
for v in "$@"; do
  if [ "$v" = base ]; then cp gpurun_out/libvosk_base.so vosk-api_amd/vosk/libvosk.so
  else cp build_exp/$v/libvosk.so vosk-api_amd/vosk/libvosk.so; fi
  timeout -k 10 300 python bench.py --workload engine --steps 20 --no-cpu-baseline --no-single-stream \
    > gpurun_out/exp_$v.json 2> gpurun_out/exp_$v.err
  python -c "
import json; d=json.load(open('gpurun_out/exp_$v.json'))
print('$v', d['value'], d['stages_ms_per_step'], d['roofline']['avg_launch_ms'])"
done
cp gpurun_out/libvosk_base.so vosk-api_amd/vosk/libvosk.so
rm -f gpurun_out/libvosk_base.so
