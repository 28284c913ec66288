"""Timeline of the last dagpu_extend_shares call of each mode in a rocprofv3
kernel + memory-copy trace of tools/single_trace.py.  Calls are separated by
gaps > 30 us between activities; the modes by the 50 ms sleep.
usage: single_timeline.py <trace dir>"""
import csv
import glob
import sys


def load(d):
    ev = []
    for f in glob.glob(f"{d}/**/*kernel_trace.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            ev.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]),
                       r["Kernel_Name"].split("(")[0].replace("dagpu::", "").replace("void ", "")[:40]))
    for f in glob.glob(f"{d}/**/*memory_copy_trace.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            size = r.get("Bytes") or r.get("Size") or "?"
            ev.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]),
                       f"copy {r.get('Direction', r.get('Operation', '?'))} {size} B"))
    ev.sort()
    return ev


def main():
    ev = load(sys.argv[1])
    # group into calls: a new call starts after a gap > 30 us with nothing running
    calls, cur, end = [], [], 0
    for e in ev:
        if cur and e[0] - end > 30_000:
            calls.append(cur)
            cur = []
        cur.append(e)
        end = max(end, e[1])
    if cur:
        calls.append(cur)
    # modes: the longest gap splits them
    gaps = [(calls[i + 1][0][0] - max(x[1] for x in calls[i]), i) for i in range(len(calls) - 1)]
    split = max(gaps)[1] if gaps else len(calls) - 1
    for name, c in (("roots_only", calls[split]), ("with_eds", calls[-1])):
        t0 = c[0][0]
        span = (max(x[1] for x in c) - t0) / 1e3
        print(f"== {name}: device span {span:.1f} us, {len(c)} activities")
        for s, e, n in c:
            print(f"{(s - t0) / 1e3:9.1f} {(e - t0) / 1e3:9.1f} {(e - s) / 1e3:8.1f}  {n}")


if __name__ == "__main__":
    main()
