# Round-2 baseline: the round-1 decoder on the large graphs (gpurun helper).
set -e
mkdir -p gpurun_out
export TMPDIR=${TMPDIR:-/tmp}
M=$TMPDIR/vamd_models
mkdir -p $M
python vosk-api_amd/tools/make_synth_model.py $M/bigram_2m --preset bigram_2m > gpurun_out/r02b_gen.log 2>&1
python vosk-api_amd/tools/make_synth_model.py $M/la_small_en_us --preset la_small_en_us >> gpurun_out/r02b_gen.log 2>&1
for m in bigram_2m la_small_en_us; do
  VOSK_AMD_DEC_PROFILE=1 timeout -k 10 300 python bench.py --model $M/$m --streams 256 --steps 20 --warmup 5 \
    --no-cpu-baseline --no-single-stream > gpurun_out/r02b_$m.json 2> gpurun_out/r02b_$m.err
  tail -c 2500 gpurun_out/r02b_$m.json
done
