"""Summarise a `tools/gpu_check.sh profile` output directory into profiles/.

    python tools/rocprof_summary.py --dir gpurun_out/r01 --tag r01

Inputs under --dir (rocprofv3 csv):
  bench_kt/**/kt_kernel_stats.csv   kernel-trace --stats of `python bench.py ...`
  fwd_kt/**/kt_kernel_trace.csv     kernel trace of tools/pmc_forward.py (plain forwards)
  fetch/**/p_counter_collection.csv --pmc FETCH_SIZE pass (same driver)
  write/**/p_counter_collection.csv --pmc WRITE_SIZE pass (same driver)
  names.json                        launch names in forward order, batch
  bench.log                         the bench JSON line (for the agreement check)

The library's dispatches (mangled `_ZN2pa...`) are cut into forwards of len(names)
launches, which maps every dispatch to its launch index.  HBM bytes per launch follow
MI355X_MICROARCH.md "HBM": FETCH_SIZE / WRITE_SIZE are KiB; on gfx950 FETCH_SIZE counts
half the bytes of a wide (16 B/lane) coalesced read, so it is doubled; WRITE_SIZE is
exact for 16-B stores.  Infinity-Cache hits are included by these memory-side counters.
Writes profiles/<tag>_summary.md, profiles/<tag>_kernel_stats.csv and updates
profiles/pmc_traffic.json (read by bench.py's roofline.traffic).
"""
import argparse
import csv
import glob
import json
import os
import shutil
import statistics
from collections import defaultdict, Counter

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def find(d, pattern):
    hits = sorted(glob.glob(os.path.join(d, "**", pattern), recursive=True))
    return hits[0] if hits else None


def ours(name):
    return name.startswith("_ZN2pa") or name.startswith("pa::") or "void pa::" in name


def forwards(rows, n):
    """rows: [(kernel, value)] in dispatch order (library kernels only) -> list of
    forwards, each a list of n (kernel, value); trailing partial forwards dropped."""
    return [rows[i:i + n] for i in range(0, len(rows) - n + 1, n)]


def trace_rows(path):
    out = []
    for r in csv.DictReader(open(path)):
        if ours(r["Kernel_Name"]):
            out.append((int(r["Dispatch_Id"]), r["Kernel_Name"],
                        (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3))
    out.sort()
    return [(k, v) for _, k, v in out]


def pmc_rows(path, counter):
    out = {}
    for r in csv.DictReader(open(path)):
        if r["Counter_Name"] == counter and ours(r["Kernel_Name"]):
            d = int(r["Dispatch_Id"])
            out[d] = (r["Kernel_Name"], out.get(d, (None, 0.0))[1] + float(r["Counter_Value"]))
    return [out[d] for d in sorted(out)]


def per_launch(fw, n, skip=1):
    """median over forwards (after `skip` warm-ups) of each launch's value; symbol per launch."""
    body = fw[skip:] if len(fw) > skip else fw
    syms = [body[0][i][0] for i in range(n)]
    for f in body:
        assert [k for k, _ in f] == syms, "dispatch sequence is not a whole number of identical forwards"
    return syms, [statistics.median(f[i][1] for f in body) for i in range(n)]


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--dir", required=True)
    p.add_argument("--tag", required=True)
    a = p.parse_args()
    out = os.path.join(ROOT, "profiles")
    os.makedirs(out, exist_ok=True)
    meta = json.load(open(os.path.join(a.dir, "names.json")))
    names, B, prec = meta["names"], meta["batch"], meta["precision"]
    n = len(names)
    lines = [f"# rocprofv3 summary {a.tag} ({prec}, batch {B})", ""]

    syms = None
    kt = find(os.path.join(a.dir, "fwd_kt"), "*kernel_trace.csv")
    dur = None
    if kt:
        syms, dur = per_launch(forwards(trace_rows(kt), n), n)
    fetch = find(os.path.join(a.dir, "fetch"), "*counter_collection.csv")
    write = find(os.path.join(a.dir, "write"), "*counter_collection.csv")
    fb = wb = None
    if fetch and write:
        s1, fb = per_launch(forwards(pmc_rows(fetch, "FETCH_SIZE"), n), n)
        s2, wb = per_launch(forwards(pmc_rows(write, "WRITE_SIZE"), n), n)
        assert s1 == s2 and (syms is None or s1 == syms)
        syms = syms or s1
        fb = [2 * 1024 * v for v in fb]
        wb = [1024 * v for v in wb]

    lines += ["## Per launch (tools/pmc_forward.py: plain forwards, median over forwards)", "",
              "| # | launch | kernel-trace us | FETCH_SIZE x2 MB | WRITE_SIZE MB | HBM MB |", "|---|---|---|---|---|---|"]
    for i, nm in enumerate(names):
        d = f"{dur[i]:.2f}" if dur else "-"
        f = f"{fb[i] / 1e6:.2f}" if fb else "-"
        w = f"{wb[i] / 1e6:.2f}" if wb else "-"
        t = f"{(fb[i] + wb[i]) / 1e6:.2f}" if fb else "-"
        lines.append(f"| {i:02d} | {nm} | {d} | {f} | {w} | {t} |")
    if dur:
        lines += ["", f"Sum of launch medians: {sum(dur):.1f} us per forward of {B} frames.", ""]

    # symbol -> launch names (for the bench stats table)
    sym_names = defaultdict(set)
    if syms:
        for s, nm in zip(syms, names):
            sym_names[s].add(nm)
    stats = find(os.path.join(a.dir, "bench_kt"), "*kernel_stats.csv")
    if stats:
        shutil.copy(stats, os.path.join(out, f"{a.tag}_kernel_stats.csv"))
        lines += ["## kernel-trace --stats of the bench command (`python bench.py`)", "",
                  "| kernel symbol | launch(es) | calls | avg us | % |", "|---|---|---|---|---|"]
        for r in csv.DictReader(open(stats)):
            nm = ",".join(sorted(sym_names.get(r["Name"], []))) or "-"
            lines.append(f"| `{r['Name'][:90]}` | {nm} | {r['Calls']} | {float(r['AverageNs']) / 1e3:.2f} | "
                         f"{float(r['Percentage']):.2f} |")
        lines.append("")
    blog = os.path.join(a.dir, "bench.log")
    if os.path.exists(blog):
        js = [ln for ln in open(blog) if ln.startswith("{")]
        if js:
            line = json.loads(js[-1])
            roof = line.get("roofline") or {}
            lines += ["## bench.py line", "", "```", js[-1].strip(), "```", ""]
            if dur and roof.get("kernel"):
                idx = [i for i, nm in enumerate(names) if nm == roof["kernel"]]
                rp = sum(dur[i] for i in idx) / len(idx)
                line_ = (f"Agreement: bench roofline kernel `{roof['kernel']}` avg {roof['avg_ms'] * 1e3:.2f} us per "
                         f"launch (HIP events, back-to-back reps)")
                btr = find(os.path.join(a.dir, "bench_kt"), "*kernel_trace.csv")
                ftr = find(os.path.join(a.dir, "fwd_kt"), "*kernel_trace.csv")
                if btr and ftr and syms:
                    # the bench command also runs these kernels at other batches (configs[2]'s
                    # 1,024-frame chunks, the streaming leg's 3-frame ticks), so --stats' per-symbol
                    # average mixes batch sizes: keep the dispatches whose grid is the one the
                    # plain B-frame forwards launch
                    grid = defaultdict(Counter)
                    for r in csv.DictReader(open(ftr)):
                        grid[r["Kernel_Name"]][r["Grid_Size_X"]] += 1
                    per = defaultdict(list)
                    for r in csv.DictReader(open(btr)):
                        g = grid.get(r["Kernel_Name"])
                        if g and r["Grid_Size_X"] == g.most_common(1)[0][0]:
                            per[r["Kernel_Name"]].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
                    if all(syms[i] in per for i in idx):
                        st = sum(statistics.median(per[syms[i]]) for i in idx) / len(idx)
                        n = sum(len(per[syms[i]]) for i in idx)
                        line_ += (f"; rocprofv3 --kernel-trace of the same bench command, median over its {n} "
                                  f"dispatches of the kernel at the B = {B} grid: {st:.2f} us")
                line_ += f"; kernel trace of plain forwards (cold-er caches): {rp:.2f} us."
                lines.append(line_)
    # fp16x3 parity-mode forwards (tools/pmc_forward.py --precision fp16x3 --out DIR/x3)
    x3n = os.path.join(a.dir, "x3", "names.json")
    x3t = find(os.path.join(a.dir, "x3_kt"), "*kernel_trace.csv")
    if os.path.exists(x3n) and x3t:
        xm = json.load(open(x3n))
        xn = xm["names"]
        _, xd = per_launch(forwards(trace_rows(x3t), len(xn)), len(xn))
        lines += ["## fp16x3 parity mode: per launch (kernel trace of plain forwards, median)", "",
                  "| # | launch | us |", "|---|---|---|"]
        lines += [f"| {i:02d} | {nm} | {d:.2f} |" for i, (nm, d) in enumerate(zip(xn, xd))]
        lines += ["", f"Sum: {sum(xd):.1f} us per forward of {xm['batch']} frames.", ""]
    fst = find(os.path.join(a.dir, "fac_kt"), "*kernel_stats.csv")
    if fst:
        lines += ["## factor path (tools/factor_prof.py: 1000 x 24 linearize + GN step)", "",
                  "| kernel | calls | avg us |", "|---|---|---|"]
        for r in csv.DictReader(open(fst)):
            if ours(r["Name"]) or r["Name"].startswith("pa::") or "pa::" in r["Name"]:
                lines.append(f"| `{r['Name'][:70]}` | {r['Calls']} | {float(r['AverageNs']) / 1e3:.2f} |")
        lines.append("")
    if fb:
        tf = os.path.join(out, "pmc_traffic.json")
        allt = json.load(open(tf)) if os.path.exists(tf) else {}
        allt = {k: v for k, v in allt.items() if isinstance(v, dict) and "bytes_per_launch" in v}
        allt[prec] = {"batch": B, "names": names, "csrc": meta.get("csrc"), "symbols": syms,
                      "bytes_per_launch": [round(f + w) for f, w in zip(fb, wb)],
                      "fetch_bytes": [round(f) for f in fb], "write_bytes": [round(w) for w in wb],
                      "source": f"profiles/{a.tag}_summary.md: rocprofv3 --pmc FETCH_SIZE / --pmc WRITE_SIZE "
                                f"(separate passes) over tools/pmc_forward.py, FETCH x2 (gfx950), median over forwards"}
        json.dump(allt, open(tf, "w"), indent=1)
    with open(os.path.join(out, f"{a.tag}_summary.md"), "w") as fh:
        fh.write("\n".join(lines) + "\n")
    print("\n".join(lines))


if __name__ == "__main__":
    main()
