set -e
mkdir -p gpurun_out
for p in 4 8; do
  VOSK_AMD_IV_PARTS=$p timeout -k 10 300 bash tools/iv_trace.sh > gpurun_out/accdev_$p.txt 2>&1
  echo "parts $p: $(grep acc_kernel gpurun_out/accdev_$p.txt)"
  VOSK_AMD_IV_PARTS=$p timeout -k 10 300 python bench.py --no-cpu-baseline --steps 40 --warmup 5 > gpurun_out/b_parts$p.json 2>/dev/null
  python3 -c "import json; d=json.load(open('gpurun_out/b_parts$p.json')); print(d['stages_ms_per_step'], d['value'])"
done
