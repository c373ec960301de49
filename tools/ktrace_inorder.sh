# Per-dispatch kernel trace of the in-order (no pipeline) bench (gpurun helper)
set -e
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace -d $GRAFT_REPO_ROOT/gpurun_out/ktrace_io -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --steps 6 --warmup 2 --no-cpu-baseline --no-pipeline > $GRAFT_REPO_ROOT/gpurun_out/ktrace_io.log 2>&1
