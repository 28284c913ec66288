"""Summarise a tools/gpu_pmc_gf16.sh run (gpurun_out/p16/<workload>/...):
kernel-trace stats and SQ / GRBM counters per launch of the GF(2^16) and
decoder kernels.  Prints the text summary and, with --json TAG, merges the
per-kernel figures into profiles/pmc_stress.json (read by bench.py's stress
rooflines), each entry tagged with TAG (the round / build the counters came from).
    python3 tools/pmc_stress.py [--json TAG] workload ...
valu_per_clk_per_cu = SQ_INSTS_VALU / (GRBM_GUI_ACTIVE / 8 XCDs) / 256 CUs;
wait_inst_frac = SQ_WAIT_INST_ANY / SQ_WAVE_CYCLES (both quad-cycle counters)."""
import collections
import csv
import glob
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
KEEP = ("leo16", "errloc", "decode128", "leo8_encode_sliced2", "repair_plan", "leo16w")


def kname(n: str) -> str:
    return n.replace("(anonymous namespace)::", "").split("(")[0].replace("void ", "").replace("dagpu::", "")


def summarise(wl: str, out: dict) -> None:
    base = os.path.join(ROOT, "gpurun_out", "p16", wl)
    print(f"== {wl}")
    s = glob.glob(f"{base}/trace/**/*kernel_stats.csv", recursive=True)
    if s:
        for r in list(csv.DictReader(open(s[0])))[:14]:
            print(f"  stats {kname(r['Name'])[:70]:70s} calls {r['Calls']:>5s} "
                  f"avg_ms {float(r['AverageNs']) / 1e6:.4f} pct {float(r['Percentage']):.1f}")
    agg = collections.defaultdict(lambda: collections.defaultdict(list))
    for p in glob.glob(f"{base}/*/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(p)):
            n = kname(r["Kernel_Name"])
            if any(x in n for x in KEEP):
                agg[n][r["Counter_Name"]].append(float(r["Counter_Value"]))
    for n, d in sorted(agg.items()):
        a = {c: sum(v) / len(v) for c, v in d.items()}
        cyc = a.get("GRBM_GUI_ACTIVE", 0) / 8
        valu = a.get("SQ_INSTS_VALU", 0)
        e = {c: round(v) for c, v in a.items()}
        if cyc and valu:
            e["valu_per_clk_per_cu"] = round(valu / cyc / 256, 3)
        if a.get("SQ_WAVE_CYCLES"):
            e["wait_inst_frac"] = round(a.get("SQ_WAIT_INST_ANY", 0) / a["SQ_WAVE_CYCLES"], 3)
            e["wait_any_frac"] = round(a.get("SQ_WAIT_ANY", 0) / a["SQ_WAVE_CYCLES"], 3)
        print(f"  pmc {n[:80]} {e}")
        # the busiest launches decide: keep the workload whose launch issued the most
        if "valu_per_clk_per_cu" in e and (n not in out or valu > out[n]["sq_insts_valu_per_launch"]):
            out[n] = {"valu_per_clk_per_cu": e["valu_per_clk_per_cu"], "wait_inst_frac": e.get("wait_inst_frac"),
                      "sq_insts_valu_per_launch": valu, "grbm_gui_active_per_launch": a.get("GRBM_GUI_ACTIVE"),
                      "workload": wl}


def main(argv):
    tag = None
    if argv[:1] == ["--json"]:
        tag, argv = argv[1], argv[2:]
    out = {}
    for wl in argv:
        summarise(wl, out)
    if tag:
        path = os.path.join(ROOT, "profiles", "pmc_stress.json")
        old = json.load(open(path)) if os.path.exists(path) else {}
        for n, e in out.items():
            e["tag"] = tag
            old[n] = e
        json.dump(old, open(path, "w"), indent=1, sort_keys=True)
        print(f"wrote {path} ({len(out)} kernels, tag {tag})")


if __name__ == "__main__":
    main(sys.argv[1:])
