# i-vector kernels of one step from a short kernel trace (gpurun helper)
set -e
bash tools/kernel_trace.sh
python3 - <<'PY'
import csv
rows = list(csv.DictReader(open('gpurun_out/ktrace/run_kernel_trace.csv')))
seq = [(r['Kernel_Name'][:44], (int(r['End_Timestamp']) - int(r['Start_Timestamp'])) / 1000) for r in rows]
idx = [i for i, x in enumerate(seq) if 'decode_kernel' in x[0]]
for x in seq[idx[-2]:idx[-1] + 1]:
    if 'stream_kernel' not in x[0]:
        print("%-44s %8.1f us" % x)
PY
