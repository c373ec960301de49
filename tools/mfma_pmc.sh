# MFMA busy cycles per kernel (one PMC pass; gpurun helper):
#   SQ_VALU_MFMA_BUSY_CYCLES and GRBM_GUI_ACTIVE over the in-order bench
#   usage: bash tools/mfma_pmc.sh <tag>
set -e
TAG=${1:-r01}
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/mfma_$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 300 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE -d $OUT -o run --output-format csv -- python3 $R/bench.py --no-cpu-baseline --no-single-stream --no-pipeline --steps 10 --warmup 2 > $OUT/bench.json 2> $OUT/err.log
ls $OUT
