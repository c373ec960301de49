"""Per-kernel FETCH_SIZE / WRITE_SIZE (bytes, averaged over launches) of the
calibration run against the known byte counts (tools/calib/fetch_calib.hip)."""
import csv
import glob
import json
import os
import sys

out = sys.argv[1]
known = json.load(open(os.path.join(out, "bytes.json")))


def per_kernel(sub, counter):
    acc = {}
    for f in glob.glob(os.path.join(out, sub, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            if r.get("Counter_Name") != counter:
                continue
            k = r["Kernel_Name"].split("(")[0].replace("void ", "").strip()
            a = acc.setdefault(k, [0.0, set()])
            a[0] += float(r["Counter_Value"]) * 1024  # KB -> bytes
            a[1].add(r["Dispatch_Id"])
    return {k: v[0] / len(v[1]) for k, v in acc.items()}


fetch, write = per_kernel("fetch", "FETCH_SIZE"), per_kernel("write", "WRITE_SIZE")
res = {"known": known, "fetch_size_bytes": fetch, "write_size_bytes": write, "ratios": {}}
for k, kb in (("stream_read", "stream_read_bytes"), ("gather16", "gather16_bytes")):
    if k in fetch:
        res["ratios"][k + ": FETCH_SIZE / algorithmic bytes"] = fetch[k] / known[kb]
        if k == "gather16":
            res["ratios"]["gather16: FETCH_SIZE per line touched"] = fetch[k] / known["gather16_lines"]
for k, kb in (("scatter4", "scatter4_bytes"), ("scatter16", "scatter16_bytes")):
    if k in write:
        res["ratios"][k + ": WRITE_SIZE / algorithmic bytes"] = write[k] / known[kb]
        res["ratios"][k + ": WRITE_SIZE per line touched"] = write[k] / known[k + "_lines"]
print(json.dumps(res, indent=1))
