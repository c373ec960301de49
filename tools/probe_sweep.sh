# LDS probe-limit sweep of the decoder on the lookahead model (gpurun helper)
set -e
mkdir -p gpurun_out
export TMPDIR=${TMPDIR:-/tmp}
M=$TMPDIR/vamd_models
mkdir -p $M
python vosk-api_amd/tools/make_synth_model.py $M/la_small_en_us --preset la_small_en_us > gpurun_out/ps_gen.log 2>&1
for p in 8 32 128 4096; do
  VOSK_AMD_DEC_LDS_PROBE=$p VOSK_AMD_DEC_PROFILE=1 timeout -k 10 300 python bench.py --model $M/la_small_en_us --streams 256 --steps 10 --warmup 3 \
    --no-cpu-baseline --no-single-stream > gpurun_out/ps_$p.json 2> gpurun_out/ps_$p.err
  echo probe $p; tail -c 1200 gpurun_out/ps_$p.json
done
