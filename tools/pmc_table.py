"""Per-launch SQ counter table from `tools/gpu_check.sh sq` output (plain forwards of
tools/pmc_forward.py; launch index from names.json):

    python tools/pmc_table.py gpurun_out/<tag>
"""
import json
import os
import statistics
import sys
from collections import defaultdict

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from rocprof_summary import find, forwards, ours  # noqa: E402
import csv  # noqa: E402


def rows(path):
    per = defaultdict(dict)
    names = {}
    for r in csv.DictReader(open(path)):
        if not ours(r["Kernel_Name"]):
            continue
        d = int(r["Dispatch_Id"])
        per[d][r["Counter_Name"]] = per[d].get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
        names[d] = r["Kernel_Name"]
    return [(names[d], per[d]) for d in sorted(per)]


def main():
    d = sys.argv[1]
    meta = json.load(open(os.path.join(d, "names.json")))
    names = meta["names"]
    n = len(names)
    acc = defaultdict(lambda: defaultdict(list))
    for sub in ("sq1", "sq2", "sq3", "fetch", "write"):
        f = find(os.path.join(d, sub), "*counter_collection.csv")
        if not f:
            continue
        for fw in forwards(rows(f), n)[1:]:
            for i, (_, cs) in enumerate(fw):
                for c, v in cs.items():
                    acc[i][c].append(v)
    med = {i: {c: statistics.median(v) for c, v in cs.items()} for i, cs in acc.items()}
    print(f"{'#':>2} {'launch':20s} {'MFMAbusy':>8s} {'waitany%':>8s} {'waitinst%':>9s} {'active%':>7s} "
          f"{'waitLDS%':>8s} {'ldsconf':>7s} {'LDS/MFMA':>8s} {'waves':>6s} {'cyc/wave':>8s}")
    for i in range(n):
        c = med.get(i, {})
        if "SQ_WAVE_CYCLES" not in c:
            continue
        wc = c["SQ_WAVE_CYCLES"]
        gui = c.get("GRBM_GUI_ACTIVE", 1)
        mf = c.get("SQ_VALU_MFMA_BUSY_CYCLES", 0)
        waves = c.get("SQ_WAVES", 0)
        # MFMA busy cycles are summed over the 1024 SIMDs, SQ_BUSY_CYCLES over the 32 shader engines
        # (tools/mfma_counters.py; GRBM_GUI_ACTIVE reads high on dispatches this short)
        sqb = c.get("SQ_BUSY_CYCLES", 8 * gui) / 32
        print(f"{i:2d} {names[i]:20s} {mf / max(1024 * sqb, 1):8.3f} {100 * c['SQ_WAIT_ANY'] / wc:8.1f} "
              f"{100 * c['SQ_WAIT_INST_ANY'] / wc:9.1f} {100 * c['SQ_ACTIVE_INST_ANY'] / wc:7.1f} "
              f"{100 * c.get('SQ_WAIT_INST_LDS', 0) / wc:8.1f} "
              f"{c.get('SQ_LDS_BANK_CONFLICT', 0) / max(c.get('SQ_LDS_IDX_ACTIVE', 1), 1):7.3f} "
              f"{c.get('SQ_INSTS_LDS', 0) / max(c.get('SQ_INSTS_MFMA', 1), 1):8.2f} {waves:6.0f} "
              f"{wc / max(waves, 1):8.0f}")
    print("raw medians:")
    for i in range(n):
        print(i, names[i], {k: round(v) for k, v in med.get(i, {}).items()})


if __name__ == "__main__":
    main()
