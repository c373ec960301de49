# full GPU suite, then the driver's bench line (gpurun helper): r03_suite_bench.sh TAG
TAG=${1:-sb}
mkdir -p gpurun_out
export TMPDIR=${TMPDIR:-/tmp}
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/suite_$TAG.log 2>&1
rc=$?
tail -4 gpurun_out/suite_$TAG.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 500 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err
rc=$?
python3 -c "import json; d=json.loads(open('gpurun_out/bench_$TAG.json').read().strip().splitlines()[-1]); print(d['value'], d['finish_ms'], json.dumps(d['result_production']))"
exit $rc
