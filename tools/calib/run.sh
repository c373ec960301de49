# FETCH_SIZE / WRITE_SIZE calibration (gpurun helper; build first:
#   hipcc -O3 --offload-arch=gfx950 tools/calib/fetch_calib.hip -o tools/calib/fetch_calib)
set -e
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/calib
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 120 $R/tools/calib/fetch_calib > $OUT/bytes.json
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d $OUT/fetch -o run --output-format csv -- $R/tools/calib/fetch_calib > /dev/null
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d $OUT/write -o run --output-format csv -- $R/tools/calib/fetch_calib > /dev/null
python3 $R/tools/calib/summary.py $OUT | tee $OUT/calib.json
