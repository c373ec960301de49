# batch-result GPU tests, then the driver's bench line (gpurun helper): r03_seg.sh TAG
TAG=${1:-seg}
mkdir -p gpurun_out
export TMPDIR=${TMPDIR:-/tmp}
timeout -k 10 700 python -u -m pytest tests/test_lattice_gpu.py tests/test_final_prune_gpu.py tests/test_api_gpu.py tests/test_batch_endpoint_gpu.py tests/test_scale_gpu.py tests/test_lookahead_gpu.py -x -v --timeout 300 --timeout-method thread > gpurun_out/seg_$TAG.log 2>&1
rc=$?
tail -3 gpurun_out/seg_$TAG.log
[ $rc -ne 0 ] && exit $rc
VOSK_AMD_STEP_PROFILE=1 timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err
rc=$?
python3 -c "import json; d=json.loads(open('gpurun_out/bench_$TAG.json').read().strip().splitlines()[-1]); print(d['value'], d['finish_ms'], d['p50_chunk_latency_ms'], json.dumps(d['result_production']))"
exit $rc
