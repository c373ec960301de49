set -e
mkdir -p gpurun_out
for m in 0 1 2 3; do
  VOSK_AMD_IV_ACC_DEV=$m timeout -k 10 300 bash tools/iv_trace.sh > gpurun_out/accdev_$m.txt 2>&1
  echo "mode $m: $(grep acc_kernel gpurun_out/accdev_$m.txt)"
done
