# silence-weighting GPU tests (new negative-delta case), default bench with CPU
# baseline, round profile (gpurun helper)
set -e
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_silence_weighting_gpu.py -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/sw_tests.log 2>&1
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
bash tools/round_bench.sh r01d
