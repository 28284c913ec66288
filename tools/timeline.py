"""Summarise a rocprofv3 kernel_trace.csv of bench.py: the DA kernels of one
timed step as a timeline relative to its first dispatch.  Steps run back to
back; with S pipeline slices a step is S x (2 RS + leaves + tree levels + DAH)
dispatches.  Usage: timeline.py kernel_trace.csv [step index, default 1 of the
timed run] [dispatches per step, default 48 = 4 slices at k = 128]"""
import csv
import sys

rows = []
with open(sys.argv[1]) as f:
    for r in csv.DictReader(f):
        n = r["Kernel_Name"]
        if "dagpu" not in n:
            continue
        rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]),
                     n.split("(")[0].replace("dagpu::", "").replace("void ", ""), r.get("Queue_Id", "")))
rows.sort()
step = int(sys.argv[2]) if len(sys.argv) > 2 else 2
per = int(sys.argv[3]) if len(sys.argv) > 3 else 48
seg = rows[step * per:(step + 1) * per]
if not seg:
    n_steps = len(rows) // per if per else 0
    sys.exit(f"step {step} is past the trace: {len(rows)} DA dispatches = {n_steps} steps of {per}")
t0 = seg[0][0]
end = max(r[1] for r in seg)
busy = {}
for s, e, n, q in seg:
    busy[n] = busy.get(n, 0) + (e - s)
print(f"step {step}: span {(end - t0) / 1e6:.3f} ms, {len(seg)} dispatches; summed kernel ms: "
      + ", ".join(f"{k} {v / 1e6:.3f}" for k, v in sorted(busy.items())))
for s, e, n, q in seg:
    print(f"{(s - t0) / 1e6:8.3f} {(e - t0) / 1e6:8.3f} {(e - s) / 1e6:7.3f}  q{q:>3} {n[:48]}")
