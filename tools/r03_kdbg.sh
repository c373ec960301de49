# Kaldi-order flat-model test under decoder debug variants (gpurun helper)
mkdir -p gpurun_out
export TMPDIR=${TMPDIR:-/tmp}
for D in 0 2 4 6; do
  VOSK_AMD_DEC_DEBUG=$D timeout -k 10 300 python -u -m pytest tests/test_kaldi_order_gpu.py -k flat -x -q -s --timeout 250 --timeout-method thread > gpurun_out/kdbg_$D.log 2>&1
  echo "debug=$D rc=$?"; grep -E "first token-count|passed|failed" gpurun_out/kdbg_$D.log | head -5
done
