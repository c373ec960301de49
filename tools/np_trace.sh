# Per-dispatch kernel durations of one non-pipelined step (gpurun helper)
set -e
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace -d $GRAFT_REPO_ROOT/gpurun_out/ktrace_np -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --steps 6 --warmup 2 --no-cpu-baseline --no-pipeline > $GRAFT_REPO_ROOT/gpurun_out/ktrace_np.log 2>&1
cd $GRAFT_REPO_ROOT
python3 - <<'PY'
import csv
rows = list(csv.DictReader(open('gpurun_out/ktrace_np/run_kernel_trace.csv')))
seq = [(r['Kernel_Name'][:44], (int(r['End_Timestamp']) - int(r['Start_Timestamp'])) / 1000, int(r['Start_Timestamp']), int(r['End_Timestamp'])) for r in rows]
idx = [i for i, x in enumerate(seq) if 'decode_kernel' in x[0]]
step = seq[idx[-2] + 1:idx[-1] + 1]
for x in step:
    print("%-44s %8.1f us  gap-before %6.1f" % (x[0], x[1], 0.0))
t0 = step[0][2]; t1 = step[-1][3]
busy = sum(x[1] for x in step)
print("step wall %.1f us, kernel busy %.1f us" % ((t1 - t0) / 1000, busy))
PY
