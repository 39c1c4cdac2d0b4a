"""Timing of pa_trajectory_linearize's workgroup kinds (1000 x 24): the whole launch, the
dynamics workgroups alone and the projection / constant-velocity workgroups alone
(pa_debug_trajectory_linearize modes 0 / 1 / 2), HIP events over `--reps` back-to-back
launches, median of 5 passes.

    python3 tools/traj_exp.py
"""
import argparse
import ctypes as C
import json
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--T", type=int, default=1000)
    p.add_argument("--L", type=int, default=24)
    p.add_argument("--reps", type=int, default=50)
    p.add_argument("--trace", action="store_true", help="per-wave phase stamps of one launch")
    a = p.parse_args()
    import torch

    from perseus_amd import _lib, pipeline, synth

    dev = torch.device("cuda", 0)
    tr = synth.synthetic_trajectories(1, a.T, a.L)
    y = torch.as_tensor(tr["y"], device=dev)
    args, out = pipeline.prepare_trajectories(y, tr["poses"], tr["vels"], tr["angvels"], tr["corners"], tr["K"],
                                              T=a.T, L=a.L, dt=1 / 12, proj_sigmas=[1.0, 1.0], dyn_sigmas=[0.1] * 6,
                                              cv_sigmas=[0.1] * 3)
    lib = _lib.lib()
    st = _lib.stream_of(dev)
    res = {}
    for mode in (0, 1, 2, 0):
        passes = []
        for _ in range(5):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            for _ in range(5):
                lib.pa_debug_trajectory_linearize(C.byref(args), mode, None, st)
            e0.record()
            for _ in range(a.reps):
                _lib.check(lib.pa_debug_trajectory_linearize(C.byref(args), mode, None, st), "traj")
            e1.record()
            torch.cuda.synchronize()
            passes.append(e0.elapsed_time(e1) * 1e3 / a.reps)
        res[f"mode{mode}"] = round(statistics.median(passes), 2)
    print(json.dumps({"T": a.T, "L": a.L, "us": res}))
    if a.trace:
        trace_phases(a, args, lib, st, torch, dev)


def trace_phases(a, args, lib, st, torch, dev):
    """One traced launch (after warm-ups): per wave kind, the median / max of each phase (us)
    and of the end time, relative to the first wave's start stamp (100 MHz clock)."""
    import numpy as np

    K = 8
    nd = a.T * (a.L - 1)
    wd = (nd + 63) // 64
    wp = (a.T * a.L * K + 255) // 256
    units = wp + wd
    nwg = wd + (units + 1) // 2
    tr = torch.zeros(nwg * 2 * 8, dtype=torch.int64, device=dev)
    for _ in range(10):
        lib.pa_debug_trajectory_linearize(C.byref(args), 0, None, st)
    lib.pa_debug_trajectory_linearize(C.byref(args), 0, C.c_void_p(tr.data_ptr()), st)
    torch.cuda.synchronize()
    t = tr.cpu().numpy().reshape(nwg, 2, 8).astype(np.float64) / 100.0  # us
    t0 = t[:, :, 0][t[:, :, 0] > 0].min()
    kinds = {"dyn_w0": t[:wd, 0], "dyn_w1": t[:wd, 1]}
    uw = t[wd:].reshape(-1, 8)[:units]
    kinds["proj"] = uw[:wp]
    kinds["cv"] = uw[wp:]
    out = {}
    for name, w in kinds.items():
        d = {"start_med": np.median(w[:, 0] - t0), "start_max": np.max(w[:, 0] - t0),
             "end_med": np.median(w[:, 7] - t0), "end_max": np.max(w[:, 7] - t0)}
        for s0, s1 in ((0, 1), (1, 2), (2, 3), (3, 4), (4, 7), (0, 4), (0, 2), (2, 4)):
            ok = (w[:, s0] > 0) & (w[:, s1] > 0)
            if ok.any():
                dd = w[ok, s1] - w[ok, s0]
                d[f"p{s0}{s1}_med"] = np.median(dd)
                d[f"p{s0}{s1}_max"] = np.max(dd)
        out[name] = {k: round(float(v), 2) for k, v in d.items()}
    print(json.dumps({"trace_us": out}))


if __name__ == "__main__":
    main()
