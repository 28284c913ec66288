"""Summarise a tools/gpu_profile.sh run into profiles/.

Reads gpurun_out/prof/{trace,pmc}_<tag>* CSVs written by rocprofv3 and writes
  profiles/kernel_stats_<tag>.csv   (rocprofv3 --kernel-trace --stats summary)
  profiles/pmc_<tag>.json           (per-kernel counters, averaged per dispatch)
  profiles/pmc_traffic.json         (HBM bytes per launch, gfx950-corrected)
  profiles/pmc_valu.json            (VALU wave-instructions and GRBM_GUI_ACTIVE per launch)
HBM bytes = 2 * FETCH_SIZE + WRITE_SIZE (KiB -> bytes): on gfx950 FETCH_SIZE
reads half of a wide streaming read's bytes (MI355X_MICROARCH.md §HBM).
"""
import collections
import csv
import glob
import json
import os
import shutil
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SHORT = {
    "leo8_encode_sliced2_kernel": "rs_encode_sliced2",
    "leo8_encode_sliced_kernel": "rs_encode_sliced",
    "leo8_encode_kernel": "rs_encode",
    "leo8_decode_kernel": "decode",
    "leo8_errlocs_kernel": "errlocs",
    "nmt_leaf_kernel": "nmt_leaves",
    "nmt_level1_kernel": "nmt_trees_l1",
    "nmt_level_kernel": "nmt_trees_ln",
    "nmt_tree_kernel": "nmt_trees",
    "dah_kernel": "dah",
}


def short(name: str) -> str:
    for k, v in SHORT.items():
        if k in name:
            return v
    return name[:40]


def main(tag: str) -> None:
    src = os.path.join(ROOT, "gpurun_out", "prof")
    os.makedirs(os.path.join(ROOT, "profiles"), exist_ok=True)
    stats = os.path.join(src, f"trace_{tag}", "run_kernel_stats.csv")
    if os.path.exists(stats):
        shutil.copy(stats, os.path.join(ROOT, "profiles", f"kernel_stats_{tag}.csv"))
    agg = collections.defaultdict(lambda: collections.defaultdict(list))
    for p in glob.glob(os.path.join(src, f"pmc_{tag}_*", "run_counter_collection.csv")):
        for r in csv.DictReader(open(p)):
            if "dagpu" not in r["Kernel_Name"]:
                continue
            agg[short(r["Kernel_Name"])][r["Counter_Name"]].append(float(r["Counter_Value"]))
    out = {k: {c: sum(v) / len(v) for c, v in d.items()} for k, d in agg.items()}
    json.dump(out, open(os.path.join(ROOT, "profiles", f"pmc_{tag}.json"), "w"), indent=1)
    traffic = {}
    for k, d in out.items():
        if "FETCH_SIZE" in d and "WRITE_SIZE" in d:
            traffic[k] = {"hbm_bytes_per_launch": (2 * d["FETCH_SIZE"] + d["WRITE_SIZE"]) * 1024,
                          "fetch_size_kib": d["FETCH_SIZE"], "write_size_kib": d["WRITE_SIZE"],
                          "tag": tag}
    if traffic:
        json.dump(traffic, open(os.path.join(ROOT, "profiles", "pmc_traffic.json"), "w"), indent=1)
    # VALU wave-instructions and GRBM_GUI_ACTIVE (summed over the 8 XCDs) per launch: bench.py's
    # whole-step issue rate (instructions per step / (step time x CUs x clock))
    valu = {k: {"valu_wave_instr_per_launch": d["SQ_INSTS_VALU"],
                "grbm_gui_active_per_launch": d.get("GRBM_GUI_ACTIVE"), "tag": tag}
            for k, d in out.items() if "SQ_INSTS_VALU" in d}
    if valu:
        json.dump(valu, open(os.path.join(ROOT, "profiles", "pmc_valu.json"), "w"), indent=1)
    print(json.dumps(traffic, indent=1))


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else "r01")
