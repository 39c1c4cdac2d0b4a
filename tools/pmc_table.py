"""Per-kernel PMC table from tools/pmc_run.sh output:  python tools/pmc_table.py gpurun_out/pmc2"""
import csv
import glob
import os
import sys
from collections import defaultdict

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from rocprof_summary import short  # noqa: E402

d = sys.argv[1]
vals = defaultdict(lambda: defaultdict(list))
for f in glob.glob(os.path.join(d, "*", "p_counter_collection.csv")):
    for r in csv.DictReader(open(f)):
        k = short(r["Kernel_Name"])
        vals[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
avg = {k: {c: sum(v) / len(v) for c, v in cs.items()} for k, cs in vals.items()}
print(f"{'kernel':22s} {'MFMAbusy/wave':>13s} {'wait_any%':>9s} {'wait_inst%':>10s} {'active%':>8s} {'ldsconf/idx':>11s} {'waitLDS%':>8s} {'HBM MB':>8s}")
for k, c in sorted(avg.items()):
    if "SQ_WAVE_CYCLES" not in c:
        continue
    wc = c["SQ_WAVE_CYCLES"]
    mf = c.get("SQ_VALU_MFMA_BUSY_CYCLES", 0)
    busy = c.get("SQ_BUSY_CYCLES", 1)
    gui = c.get("GRBM_GUI_ACTIVE", 1)
    hbm = (2 * c.get("FETCH_SIZE", 0) + c.get("WRITE_SIZE", 0)) * 1024 / 1e6
    print(f"{k:22s} {mf / max(gui,1) / 1024:13.3f} {100*c['SQ_WAIT_ANY']/wc:9.1f} {100*c['SQ_WAIT_INST_ANY']/wc:10.1f} "
          f"{100*c['SQ_ACTIVE_INST_ANY']/wc:8.1f} {c.get('SQ_LDS_BANK_CONFLICT',0)/max(c.get('SQ_LDS_IDX_ACTIVE',1),1):11.3f} "
          f"{100*c.get('SQ_WAIT_INST_LDS',0)/wc:8.1f} {hbm:8.1f}")
print("raw:")
for k, c in sorted(avg.items()):
    print(k, {n: round(v) for n, v in c.items()})
