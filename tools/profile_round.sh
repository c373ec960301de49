R=$GRAFT_REPO_ROOT
ARGS="--no-cpu-baseline --no-single-stream --no-order-line --no-engine-line --steps 20 --warmup 5"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof6/trace -o run --output-format csv -- python3 $R/bench.py $ARGS > $R/gpurun_out/prof6_trace.log 2>&1 && \
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE -d $R/gpurun_out/prof6/fetch -o run --output-format csv -- python3 $R/bench.py $ARGS > $R/gpurun_out/prof6_fetch.log 2>&1 && \
timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE -d $R/gpurun_out/prof6/write -o run --output-format csv -- python3 $R/bench.py $ARGS > $R/gpurun_out/prof6_write.log 2>&1 && \
python3 $R/tools/pmc_summary.py $R/gpurun_out/prof6 > $R/gpurun_out/prof6_pmc.json
