# Batch-path GPU tests after a decoder or result-pipeline change (gpurun helper)
# usage: bash tools/batch_check.sh <tag> [pytest files...]
TAG=${1:-b}; shift
mkdir -p gpurun_out
export TMPDIR=${TMPDIR:-/tmp}
FILES=${@:-tests/test_batch_endpoint_gpu.py tests/test_batching.py tests/test_final_prune_gpu.py tests/test_segment_best_path_gpu.py}
timeout -k 10 900 python -u -m pytest $FILES -x -v --timeout 600 --timeout-method thread > gpurun_out/batch_$TAG.log 2>&1
rc=$?; tail -15 gpurun_out/batch_$TAG.log; exit $rc
