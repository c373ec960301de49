# Decoder PMC counters on the 2.4 M-state graph (gpurun helper; one counter
# pass per rocprofv3 run).  usage: bash tools/dec_pmc.sh <tag>
set -e
TAG=${1:-x}
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/decpmc_$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
M=/tmp/vamd_models
mkdir -p $M
python3 $R/vosk-api_amd/tools/make_synth_model.py $M/bigram_2m --preset bigram_2m > $OUT/gen.log 2>&1
timeout -s KILL 60 rocprofv3 --list-avail > $OUT/avail.txt 2>&1 || true
B="python3 $R/bench.py --model $M/bigram_2m --no-cpu-baseline --no-single-stream --no-pipeline --steps 4 --warmup 1"
timeout -s KILL 200 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_SMEM SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_BRANCH -d $OUT/p1 -o run --output-format csv -- $B > $OUT/b1.json 2> $OUT/e1.log
timeout -s KILL 200 rocprofv3 --pmc SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR -d $OUT/p2 -o run --output-format csv -- $B > $OUT/b2.json 2> $OUT/e2.log
timeout -s KILL 200 rocprofv3 --kernel-trace --stats -d $OUT/kt -o run --output-format csv -- $B > $OUT/b3.json 2> $OUT/e3.log
find $OUT -name "*.csv" | head -20
