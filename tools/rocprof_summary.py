"""Summarise rocprofv3 outputs into profiles/ (kernel stats + PMC HBM traffic).

    python tools/rocprof_summary.py --stats gpurun_out/prof_r1/kt_kernel_stats.csv \
        --fetch gpurun_out/pmc_fetch/f_counter_collection.csv \
        --write gpurun_out/pmc_write/w_counter_collection.csv --tag r01 [--precision fp16]

HBM bytes per launch follow MI355X_MICROARCH.md "HBM": FETCH_SIZE / WRITE_SIZE are KiB;
on gfx950 FETCH_SIZE reads half the bytes of a wide (16 B/lane) coalesced stream, so it
is doubled; WRITE_SIZE is exact for 16-B stores.  Infinity-Cache hits are counted by
these memory-side counters (the guide notes they are not excluded).
"""
import argparse
import csv
import json
import os
import re
import shutil
from collections import defaultdict

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def short(sym: str) -> str:
    m = re.search(r"conv_igemmI(DF16_|f)Li(\d+)ELi(\d+)ELi(\d)E", sym)
    if m:
        return f"conv{m.group(4)}x{m.group(4)}_{m.group(2)}x{m.group(3)}"
    for k in ("stem_kernel", "maxpool_kernel", "head_kernel", "dyn_kernel", "proj_kernel", "cv_kernel"):
        if k in sym:
            return {"stem_kernel": "stem_conv7x7", "maxpool_kernel": "maxpool", "head_kernel": "avgpool_fc"}.get(k, k)
    return sym[:60]


def pmc(path, counter):
    per = defaultdict(list)
    for r in csv.DictReader(open(path)):
        if r["Counter_Name"] != counter:
            continue
        per[short(r["Kernel_Name"])].append(float(r["Counter_Value"]))
    return per


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--stats")
    p.add_argument("--fetch")
    p.add_argument("--write")
    p.add_argument("--tag", required=True)
    p.add_argument("--precision", default="fp16")
    a = p.parse_args()
    out = os.path.join(ROOT, "profiles")
    os.makedirs(out, exist_ok=True)
    lines = [f"# rocprofv3 summary {a.tag} ({a.precision})", ""]
    if a.stats:
        shutil.copy(a.stats, os.path.join(out, f"{a.tag}_kernel_stats.csv"))
        lines += ["| kernel | calls | avg us | % |", "|---|---|---|---|"]
        for r in csv.DictReader(open(a.stats)):
            lines.append(f"| {short(r['Name'])} | {r['Calls']} | {float(r['AverageNs'])/1e3:.2f} | {r['Percentage']} |")
        lines.append("")
    if a.fetch and a.write:
        f, w = pmc(a.fetch, "FETCH_SIZE"), pmc(a.write, "WRITE_SIZE")
        traffic = {}
        lines += ["| kernel | launches | FETCH_SIZE x2 (MB/launch) | WRITE_SIZE (MB/launch) | HBM bytes/launch |",
                  "|---|---|---|---|---|"]
        for k in sorted(f):
            if k not in w:
                continue
            fb = 2 * 1024 * sum(f[k]) / len(f[k])
            wb = 1024 * sum(w[k]) / len(w[k])
            traffic[k] = fb + wb
            lines.append(f"| {k} | {len(f[k])} | {fb/1e6:.2f} | {wb/1e6:.2f} | {(fb+wb)/1e6:.2f} MB |")
        tf = os.path.join(out, "pmc_traffic.json")
        allt = json.load(open(tf)) if os.path.exists(tf) else {}
        allt[a.precision] = traffic
        allt["source"] = f"{a.tag}: rocprofv3 --pmc FETCH_SIZE / --pmc WRITE_SIZE (separate passes), FETCH x2 (gfx950)"
        json.dump(allt, open(tf, "w"), indent=1)
    with open(os.path.join(out, f"{a.tag}_summary.md"), "w") as fh:
        fh.write("\n".join(lines) + "\n")
    print("\n".join(lines))


if __name__ == "__main__":
    main()
