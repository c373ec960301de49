# decoder parity + lattice tests, then bench / phase probe (gpurun helper)
set -e
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_lattice_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/dec_tests.log 2>&1
bash tools/probe_r01.sh
