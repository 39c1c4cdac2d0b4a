"""MFMA utilisation per launch from rocprofv3 counters (north_star: "MFMA utilisation on the 3x3
blocks"), for the kernels of the current csrc digest.

    # on the GPU box (tools/gpu_check.sh mfma <tag> runs exactly this):
    rocprofv3 --pmc SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVE_CYCLES GRBM_GUI_ACTIVE \
        --output-format csv -d gpurun_out/<tag>/mfma -o p -- python3 tools/pmc_forward.py --out gpurun_out/<tag>
    # here:
    python tools/mfma_counters.py gpurun_out/<tag> --tag <tag>

Normalisation (MI355X_MICROARCH.md, "Per-instruction cycle constants" and "DVFS give-back"):
SQ_VALU_MFMA_BUSY_CYCLES is summed over every SIMD of the chip and counts shader cycles (16 per
v_mfma_f32_16x16x32_f16, 32 per 32x32x16); SQ_BUSY_CYCLES is summed over the 32 shader engines,
so SQ_BUSY_CYCLES / 32 is the launch's busy span in shader cycles (it agrees with SQ_WAVE_CYCLES
per wave x 4, the waves living the whole launch).  Hence

    fraction of the nominal peak          = MFMA_BUSY / (1024 SIMDs x duration x 2.4 GHz)
    busy fraction of the launch's cycles = MFMA_BUSY / (1024 SIMDs x SQ_BUSY_CYCLES / 32)
    clock the chip held                   = SQ_BUSY_CYCLES / 32 / duration

(the first is the same quantity as bench.py's FLOPs / (time x 2.5 PF) when the MFMAs are
16x16x32 f16: 16 cycles x 1024 FLOP/cycle/SIMD = 16,384 FLOP each; the second removes the DVFS
give-back).  GRBM_GUI_ACTIVE / 8 / duration reads 2.6-3.2 GHz on these ~20 us dispatches (the
guide: it reads high below ~0.3 ms), so it is recorded but not used.  The old
tools/pmc_table.py column divided by GRBM_GUI_ACTIVE itself (8 XCDs' worth) and read ~8x low.

Writes profiles/<tag>_mfma_counters.txt and the digest-keyed record profiles/pmc_mfma.json
(bench.py reports it as per_kernel_roofline.mfma_busy_counter when the digest matches).
"""
import argparse
import csv
import glob
import json
import os
import statistics
import sys
from collections import defaultdict

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
SIMDS = 1024        # 256 CUs x 4 SIMDs
NOMINAL_GHZ = 2.4   # the clock the 2.5 PF dense fp16 peak is quoted at
FLOP_PER_MFMA = 16 * 16 * 32 * 2
COUNTERS = ("SQ_INSTS_MFMA", "SQ_VALU_MFMA_BUSY_CYCLES", "SQ_BUSY_CYCLES", "SQ_WAVE_CYCLES", "GRBM_GUI_ACTIVE")


def ours(name):
    return name.startswith("_ZN2pa") or name.startswith("pa::") or "void pa::" in name


def dispatches(path):
    per = defaultdict(dict)
    meta = {}
    for r in csv.DictReader(open(path)):
        if not ours(r["Kernel_Name"]):
            continue
        d = int(r["Dispatch_Id"])
        per[d][r["Counter_Name"]] = per[d].get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
        meta[d] = (r["Kernel_Name"], (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
    return [(meta[d][0], meta[d][1], per[d]) for d in sorted(per)]


def summarise(rows, n, skip=1):
    """median per launch over the forwards after `skip` warm-ups"""
    fws = [rows[i:i + n] for i in range(0, len(rows) - n + 1, n)]
    body = fws[skip:] if len(fws) > skip else fws
    syms = [k for k, _, _ in body[0]]
    for f in body:
        assert [k for k, _, _ in f] == syms, "dispatch sequence is not a whole number of identical forwards"
    out = []
    for i in range(n):
        c = {k: statistics.median(f[i][2].get(k, 0.0) for f in body) for k in COUNTERS}
        c["dur_us"] = statistics.median(f[i][1] for f in body)
        out.append(c)
    return syms, out


def main():
    p = argparse.ArgumentParser()
    p.add_argument("dir")
    p.add_argument("--tag", required=True)
    a = p.parse_args()
    from bench import conv_flops

    meta = json.load(open(os.path.join(a.dir, "names.json")))
    names, B, prec = meta["names"], meta["batch"], meta["precision"]
    hits = sorted(glob.glob(os.path.join(a.dir, "mfma", "**", "*counter_collection.csv"), recursive=True))
    if not hits:
        raise SystemExit(f"no counter csv under {a.dir}/mfma")
    syms, per = summarise(dispatches(hits[0]), len(names))
    cf = conv_flops(B, fused_head=names[-1] != "avgpool_fc")
    fl = cf if prec == "fp16" and len(cf) == len(names) else [None] * len(names)
    lines = [f"# MFMA counters {a.tag} ({prec}, batch {B}; csrc {meta.get('csrc')})", "",
             "rocprofv3 --pmc SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVE_CYCLES GRBM_GUI_ACTIVE over "
             "tools/pmc_forward.py (plain forwards), median per launch over forwards; busy/nominal = "
             "MFMA_BUSY / (1024 SIMDs x dur x 2.4 GHz) (= bench.py's conv3x3_mfma_frac quantity); busy/cycles = "
             "MFMA_BUSY / (1024 x SQ_BUSY_CYCLES/32); clock = SQ_BUSY_CYCLES/32/dur; FLOP ratio = MFMA FLOPs executed / algorithmic FLOPs (padding).", "",
             "| # | launch | dur us | MFMA insts | MFMA busy cyc | cyc/MFMA | clock GHz | busy/cycles | busy/nominal "
             "| FLOP ratio |", "|---|---|---|---|---|---|---|---|---|---|"]
    rec = []
    for i, (nm, c) in enumerate(zip(names, per)):
        cyc = c["SQ_BUSY_CYCLES"] / 32  # 32 shader engines
        ghz = cyc / (c["dur_us"] * 1e3) if c["dur_us"] > 0 else 0.0
        fc = c["SQ_VALU_MFMA_BUSY_CYCLES"] / (SIMDS * cyc) if cyc else 0.0
        fn = c["SQ_VALU_MFMA_BUSY_CYCLES"] / (SIMDS * c["dur_us"] * 1e3 * NOMINAL_GHZ) if c["dur_us"] else 0.0
        cpm = c["SQ_VALU_MFMA_BUSY_CYCLES"] / c["SQ_INSTS_MFMA"] if c["SQ_INSTS_MFMA"] else 0.0
        ratio = (c["SQ_INSTS_MFMA"] * FLOP_PER_MFMA / fl[i]) if fl[i] else None
        lines.append(f"| {i:02d} | {nm} | {c['dur_us']:.2f} | {c['SQ_INSTS_MFMA']:.0f} | "
                     f"{c['SQ_VALU_MFMA_BUSY_CYCLES']:.0f} | {cpm:.1f} | {ghz:.3f} | {fc:.3f} | {fn:.3f} | "
                     f"{'-' if ratio is None else f'{ratio:.3f}'} |")
        rec.append({"launch": nm, "dur_us": round(c["dur_us"], 3), "mfma_insts": round(c["SQ_INSTS_MFMA"]),
                    "mfma_busy_cycles": round(c["SQ_VALU_MFMA_BUSY_CYCLES"]), "clock_ghz": round(ghz, 4),
                    "busy_frac_of_cycles": round(fc, 4), "busy_frac_of_nominal": round(fn, 4)})
    conv = [r for r in rec if r["launch"].startswith("conv3x3")]
    if conv:
        lines += ["", f"3x3 convs: busy/cycles {min(r['busy_frac_of_cycles'] for r in conv):.3f}-"
                      f"{max(r['busy_frac_of_cycles'] for r in conv):.3f}, busy/nominal "
                      f"{min(r['busy_frac_of_nominal'] for r in conv):.3f}-"
                      f"{max(r['busy_frac_of_nominal'] for r in conv):.3f}"]
    txt = os.path.join(ROOT, "profiles", f"{a.tag}_mfma_counters.txt")
    with open(txt, "w") as fh:
        fh.write("\n".join(lines) + "\n")
    tf = os.path.join(ROOT, "profiles", "pmc_mfma.json")
    allm = json.load(open(tf)) if os.path.exists(tf) else {}
    allm[prec] = {"batch": B, "names": names, "csrc": meta.get("csrc"), "symbols": syms, "per_launch": rec,
                  "source": f"profiles/{a.tag}_mfma_counters.txt"}
    json.dump(allm, open(tf, "w"), indent=1)
    print("\n".join(lines))


if __name__ == "__main__":
    main()
