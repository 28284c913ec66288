"""Timeline of one Repair call from a rocprofv3 kernel_trace.csv of
`bench.py --mode repair`: the dagpu kernels between two consecutive
finalize_repair_kernel dispatches (= one repair), with the gaps between them.
Usage: repair_timeline.py kernel_trace.csv [repair index, default 2]"""
import csv
import sys

rows = []
with open(sys.argv[1]) as f:
    for r in csv.DictReader(f):
        rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"].split("(")[0].replace("void ", "")))
rows.sort()
fin = [i for i, r in enumerate(rows) if "finalize_repair" in r[2]]
idx = int(sys.argv[2]) if len(sys.argv) > 2 else 2
if idx < 1 or idx >= len(fin):
    sys.exit(f"{len(fin)} repairs in the trace")
seg = rows[fin[idx - 1] + 1:fin[idx] + 1]
# before the repair: the previous call's restore_presence_kernel, then the bench's
# input restore (the damaged EDS copied back, the first copyBuffer); the repair
# starts with the dispatch after that copy
first = next(i for i, r in enumerate(seg) if "copyBuffer" in r[2]) + 1
seg = seg[first:]
t0 = seg[0][0]
busy = sum(e - s for s, e, _ in seg)
print(f"repair {idx}: span {(seg[-1][1] - t0) / 1e6:.3f} ms, kernels {busy / 1e6:.3f} ms, {len(seg)} dispatches")
prev_end = t0
for s, e, n in seg:
    gap = (s - prev_end) / 1e3
    print(f"{(s - t0) / 1e6:8.3f} {(e - s) / 1e6:7.3f}  gap {gap:7.1f} us  {n[-60:]}")
    prev_end = max(prev_end, e)
