# Decoder iteration (gpurun helper): decoder parity tests, then the large-graph
# bench lines.  usage: bash tools/r02_dec_iter.sh <tag>
set -e
TAG=${1:-x}
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_decoder_prune_gpu.py tests/test_lattice_gpu.py tests/test_gpu_parity.py tests/test_large_graph_gpu.py -x -q --timeout 300 --timeout-method thread > gpurun_out/dec_iter_$TAG.log 2>&1 || { tail -30 gpurun_out/dec_iter_$TAG.log; exit 1; }
tail -3 gpurun_out/dec_iter_$TAG.log
bash tools/r02_dec.sh $TAG
