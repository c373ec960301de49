# batch-path result tests, then the driver's bench line (gpurun helper)
TAG=${1:-p}
mkdir -p gpurun_out
export TMPDIR=${TMPDIR:-/tmp}
(while true; do sleep 50; echo "[hb] $(date +%T)" >> gpurun_out/hb_$TAG.log; done) &
HB=$!
trap "kill $HB" EXIT
timeout -k 10 900 python -u -m pytest tests/test_final_prune_gpu.py tests/test_api_gpu.py tests/test_batch_endpoint_gpu.py tests/test_batching.py tests/test_lattice_gpu.py tests/test_scale_gpu.py -x -v --timeout 600 --timeout-method thread > gpurun_out/fp_$TAG.log 2>&1
rc=$?; tail -8 gpurun_out/fp_$TAG.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 500 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/fp_bench_$TAG.json 2> gpurun_out/fp_bench_$TAG.err
rc=$?
python3 -c "import json; d=json.load(open('gpurun_out/fp_bench_$TAG.json')); print(d['value'], d['finish_ms'], d['p50_chunk_latency_ms'], d['result_production'])"
exit $rc
