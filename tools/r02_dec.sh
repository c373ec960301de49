# Decoder performance on the large graphs (gpurun helper): bench lines with
# phase clocks and the per-stream spread.  usage: bash tools/r02_dec.sh <tag>
set -e
TAG=${1:-x}
mkdir -p gpurun_out
export TMPDIR=${TMPDIR:-/tmp}
M=$TMPDIR/vamd_models
mkdir -p $M
python vosk-api_amd/tools/make_synth_model.py $M/bigram_2m --preset bigram_2m > gpurun_out/r02d_gen.log 2>&1
python vosk-api_amd/tools/make_synth_model.py $M/la_small_en_us --preset la_small_en_us >> gpurun_out/r02d_gen.log 2>&1
for m in bigram_2m la_small_en_us; do
  VOSK_AMD_DEC_PROFILE=1 timeout -k 10 300 python bench.py --model $M/$m --streams 256 --steps 20 --warmup 5 \
    --no-cpu-baseline --no-single-stream > gpurun_out/r02d_${TAG}_$m.json 2> gpurun_out/r02d_${TAG}_$m.err
  tail -c 3000 gpurun_out/r02d_${TAG}_$m.json
done
