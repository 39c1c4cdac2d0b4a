"""Per-kernel statistics from a rocprofv3 database (the .db written when no --output-format
is given): calls, average / total duration, grid, VGPRs and scratch per kernel symbol.

    python tools/rocpd_stats.py gpurun_out/<dir>/run_results.db [--top 40] [--csv out.csv]
"""
import argparse
import collections
import csv
import sqlite3


def kernel_rows(db):
    c = sqlite3.connect(db)
    names = [r[0] for r in c.execute("select name from sqlite_master where type='table'")]
    suf = next(n for n in names if n.startswith("rocpd_kernel_dispatch")).split("rocpd_kernel_dispatch")[1]
    q = (f"select s.display_name, d.end - d.start, d.grid_size_x / d.workgroup_size_x, d.grid_size_y, "
         f"s.arch_vgpr_count, s.accum_vgpr_count, s.private_segment_size "
         f"from rocpd_kernel_dispatch{suf} d join rocpd_info_kernel_symbol{suf} s on d.kernel_id = s.id")
    return list(c.execute(q))


def main():
    p = argparse.ArgumentParser()
    p.add_argument("db")
    p.add_argument("--top", type=int, default=40)
    p.add_argument("--csv")
    a = p.parse_args()
    agg = collections.OrderedDict()
    for name, ns, gx, gy, vg, ag, scr in kernel_rows(a.db):
        r = agg.setdefault(name, {"calls": 0, "total_ns": 0, "grid": f"{gx}x{gy}", "vgpr": vg, "agpr": ag, "scratch": scr})
        r["calls"] += 1
        r["total_ns"] += ns
    rows = sorted(agg.items(), key=lambda kv: -kv[1]["total_ns"])
    if a.csv:
        with open(a.csv, "w", newline="") as f:
            w = csv.writer(f)
            w.writerow(["Name", "Calls", "AverageNs", "TotalDurationNs", "Grid", "VGPR", "AGPR", "Scratch"])
            for n, r in rows:
                w.writerow([n, r["calls"], r["total_ns"] / r["calls"], r["total_ns"], r["grid"], r["vgpr"], r["agpr"],
                            r["scratch"]])
    for n, r in rows[:a.top]:
        print(f"{n[:80]:80s} {r['calls']:6d} {r['total_ns'] / r['calls'] / 1e3:8.2f} us  grid {r['grid']:>8s} "
              f"v{r['vgpr']} a{r['agpr']} s{r['scratch']}")


if __name__ == "__main__":
    main()
