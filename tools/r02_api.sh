# Batch path through the public API (gpurun helper): batch GPU tests, a short
# bench line, then the default bench.  usage: bash tools/r02_api.sh <tag> [full]
set -e
TAG=${1:-x}
mkdir -p gpurun_out
export TMPDIR=${TMPDIR:-/tmp}
timeout -k 10 900 python -u -m pytest tests/test_batch_endpoint_gpu.py tests/test_api_gpu.py \
  tests/test_lookahead_gpu.py -x -v --timeout 300 --timeout-method thread > gpurun_out/api_tests_$TAG.log 2>&1 \
  || { tail -40 gpurun_out/api_tests_$TAG.log; exit 1; }
tail -5 gpurun_out/api_tests_$TAG.log
timeout -k 10 600 python bench.py --stream-seconds 10 --no-cpu-baseline --no-single-stream \
  > gpurun_out/api_short_$TAG.json 2> gpurun_out/api_short_$TAG.err || { tail -30 gpurun_out/api_short_$TAG.err; exit 1; }
tail -c 3000 gpurun_out/api_short_$TAG.json
if [ "$2" = full ]; then
  timeout -k 10 900 python bench.py > gpurun_out/api_full_$TAG.json 2> gpurun_out/api_full_$TAG.err \
    || { tail -30 gpurun_out/api_full_$TAG.err; exit 1; }
  tail -c 4000 gpurun_out/api_full_$TAG.json
fi
