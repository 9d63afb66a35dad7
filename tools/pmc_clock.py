"""Per-kernel clock and MFMA busy from a rocprofv3 --pmc counter CSV (Start/End timestamps are in it).

    python tools/pmc_clock.py <dir with *counter_collection.csv> [kernel-substring]

clock = GRBM_GUI_ACTIVE / 8 XCDs / duration (MI355X_MICROARCH.md, DVFS give-back);
MFMA busy = SQ_VALU_MFMA_BUSY_CYCLES / (1024 SIMDs x GRBM_GUI_ACTIVE / 8)."""
import collections
import csv
import glob
import sys


def main():
    d, sub = sys.argv[1], (sys.argv[2] if len(sys.argv) > 2 else "")
    rows = collections.defaultdict(dict)
    names = {}
    for f in glob.glob(f"{d}/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            if sub not in r["Kernel_Name"]:
                continue
            k = (f, r["Dispatch_Id"])
            rows[k][r["Counter_Name"]] = float(r["Counter_Value"])
            rows[k]["_dur"] = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-9
            names[k] = r["Kernel_Name"][:60]
    agg = collections.defaultdict(list)
    for k, c in rows.items():
        agg[names[k]].append(c)
    for n, cs in agg.items():
        out = [f"{n:60s} n={len(cs)}"]
        dur = sum(c["_dur"] for c in cs) / len(cs)
        out.append(f"dur {dur * 1e6:8.1f} us")
        if "GRBM_GUI_ACTIVE" in cs[0]:
            g = sum(c["GRBM_GUI_ACTIVE"] for c in cs) / len(cs)
            out.append(f"clock {g / 8 / dur / 1e9:5.2f} GHz")
            if "SQ_VALU_MFMA_BUSY_CYCLES" in cs[0]:
                m = sum(c["SQ_VALU_MFMA_BUSY_CYCLES"] for c in cs) / len(cs)
                out.append(f"mfma busy {m / (1024 * g / 8):5.3f}")
        for key in ("SQ_WAVE_CYCLES", "SQ_ACTIVE_INST_ANY", "SQ_WAIT_INST_ANY", "SQ_WAIT_ANY"):
            if key in cs[0] and "SQ_WAVE_CYCLES" in cs[0] and key != "SQ_WAVE_CYCLES":
                out.append(f"{key[3:]} {sum(c[key] for c in cs) / sum(c['SQ_WAVE_CYCLES'] for c in cs):5.3f}")
        print("  ".join(out))


if __name__ == "__main__":
    main()
