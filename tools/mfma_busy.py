"""Per-kernel-class MFMA busy fraction and effective clock from ONE rocprofv3 --pmc pass of
GRBM_GUI_ACTIVE + SQ_VALU_MFMA_BUSY_CYCLES over the bench (MI355X_MICROARCH.md 'DVFS give-back':
clock = GRBM_GUI_ACTIVE / 8 XCDs / duration; busy = SQ_VALU_MFMA_BUSY_CYCLES / (1024 SIMDs x
GRBM_GUI_ACTIVE / 8)).  Writes `profiles/<round>_mfma_busy.json`:

    python tools/mfma_busy.py PMC_DIR OUT_JSON
"""
import collections
import csv
import glob
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from traffic import CLASSES  # noqa: E402


def main():
    d, out = sys.argv[1:3]
    disp = collections.defaultdict(dict)
    for f in glob.glob(f"{d}/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            k = (f, r["Dispatch_Id"])
            disp[k][r["Counter_Name"]] = disp[k].get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
            disp[k]["_dur"] = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-9
            disp[k]["_name"] = r["Kernel_Name"]
    agg = collections.defaultdict(lambda: [0.0, 0.0, 0.0, 0])
    for c in disp.values():
        if "GRBM_GUI_ACTIVE" not in c or "SQ_VALU_MFMA_BUSY_CYCLES" not in c:
            continue
        cls = next((cl for frag, cl in CLASSES if frag in c["_name"]), None)
        if cls is None:
            continue
        a = agg[cls]
        a[0] += c["GRBM_GUI_ACTIVE"]
        a[1] += c["SQ_VALU_MFMA_BUSY_CYCLES"]
        a[2] += c["_dur"]
        a[3] += 1
    res = {}
    for cls, (g, m, dur, n) in sorted(agg.items()):
        res[cls] = {"dispatches": n, "avg_dur_us": round(dur / n * 1e6, 1),
                    "clock_ghz": round(g / 8 / dur / 1e9, 3), "mfma_busy": round(m / (1024 * g / 8), 4)}
        print(f"{cls:45s} n={n:3d} dur {dur / n * 1e6:8.1f} us  clock {g / 8 / dur / 1e9:5.2f} GHz  "
              f"mfma busy {m / (1024 * g / 8):5.3f}")
    json.dump({"note": "rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES (one pass) over bench.py; "
                       "profiled passes run ~2-5% below the un-profiled clock",
               "kernels": res}, open(out, "w"), indent=1)


if __name__ == "__main__":
    main()
