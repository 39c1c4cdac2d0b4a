"""Interleaved timing of pa_trajectory_gn_step variants (assembler waves per trajectory,
pa_debug_gn_set_assemblers; 128: the two-ended elimination, 64: cyclic reduction) at T x 24
(default 1000 and the streaming pose stage's 3), HIP
events over back-to-back launches; outputs checked against the shipped variant's.

    python tools/gn_ab.py [--na 128 64 0] [--T 1000 3] [--rounds 5]
"""
import argparse
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--na", type=int, nargs="+", default=[128, 64, 0])
    p.add_argument("--T", type=int, nargs="+", default=[1000, 3])
    p.add_argument("--rounds", type=int, default=5)
    p.add_argument("--reps", type=int, default=20)
    a = p.parse_args()
    import torch

    from perseus_amd import _lib, pipeline, synth

    L_ = _lib.lib()
    dev = torch.device("cuda", 0)
    s = torch.cuda.current_stream(dev)
    for T, L in ((T, 24) for T in a.T):
        tr = synth.synthetic_trajectories(1, T, L)
        y = torch.as_tensor(tr["y"], device=dev)
        args, lin = pipeline.prepare_trajectories(y, tr["poses"], tr["vels"], tr["angvels"], tr["corners"], tr["K"],
                                                  T=T, L=L, dt=1 / 12, proj_sigmas=[1.0, 1.0],
                                                  dyn_sigmas=[0.1] * 6, cv_sigmas=[0.1] * 3)
        pipeline.launch(args, dev)
        plan = pipeline.GNPlan(lin, T=T, L=L, lam=1e-3)
        ref = None
        res = {na: [] for na in a.na}
        for r in range(a.rounds + 1):
            for na in a.na:
                _lib.check(L_.pa_debug_gn_set_assemblers(na))
                plan.launch()
                if r == 0:
                    d = plan.out["delta"].clone()
                    ref = d if ref is None else ref
                    print(f"T={T} L={L} na={na}: delta max |diff| vs na={a.na[0]}: "
                          f"{(d - ref).abs().max().item():.3e}, solved {(plan.out['info'] == 0).sum().item()}",
                          flush=True)
                    continue
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record(s)
                for _ in range(a.reps):
                    plan.launch()
                e1.record(s)
                torch.cuda.synchronize()
                res[na].append(e0.elapsed_time(e1) / a.reps * 1e3)
        print(f"T={T} L={L}: " + " | ".join(f"na={na} {statistics.median(v):.1f} us" for na, v in res.items()),
              flush=True)
    _lib.check(L_.pa_debug_gn_set_assemblers(0))


if __name__ == "__main__" and not os.environ.get("GN_TRACE"):
    main()


def trace(T=3, L=24, variant=0):
    """Per-frame stamps of one traced pa_trajectory_gn_step (pa_debug_gn_set_trace)."""
    import numpy as np
    import torch

    from perseus_amd import _lib, pipeline, synth

    L_ = _lib.lib()
    dev = torch.device("cuda", 0)
    tr = synth.synthetic_trajectories(1, T, L)
    y = torch.as_tensor(tr["y"], device=dev)
    args, lin = pipeline.prepare_trajectories(y, tr["poses"], tr["vels"], tr["angvels"], tr["corners"], tr["K"],
                                              T=T, L=L, dt=1 / 12, proj_sigmas=[1.0, 1.0], dyn_sigmas=[0.1] * 6,
                                              cv_sigmas=[0.1] * 3)
    pipeline.launch(args, dev)
    plan = pipeline.GNPlan(lin, T=T, L=L, lam=1e-3)
    buf = torch.zeros(T * 256, dtype=torch.int64, device=dev)
    _lib.check(L_.pa_debug_gn_set_assemblers(variant))
    for _ in range(3):
        plan.launch()
    _lib.check(L_.pa_debug_gn_set_trace(buf.data_ptr()))
    plan.launch()
    torch.cuda.synchronize()
    _lib.check(L_.pa_debug_gn_set_trace(None))
    _lib.check(L_.pa_debug_gn_set_assemblers(0))
    s = buf.cpu().numpy().reshape(T, 256).astype(np.int64)
    t0 = s[0, 0]
    if variant & 64:  # gn_cr_kernel's stamps (wave 0, 10 ns ticks)
        ns = lambda j: (s[0, j] - t0) * 10  # noqa: E731
        print(f"assembly (wave 0) {ns(2)} ns, barrier {ns(1)} ns")
        for lv in range(6):
            if s[0, 10 + 2 * lv]:
                print(f"level {lv}: eliminated {ns(10 + 2 * lv)} ns, survivors {ns(11 + 2 * lv)} ns")
        print(f"last solve {ns(30)} ns")
        for lv in range(5, -1, -1):
            if s[0, 31 + lv]:
                print(f"back level {lv}: {ns(31 + lv)} ns")
        print(f"end {ns(40)} ns")
        return
    for l in range(L):
        a0, a1 = (s[0, 2 * l] - t0) * 10, (s[0, 2 * l + 1] - t0) * 10
        w, rd, sw, dn = ((s[0, 64 + 4 * l + j] - t0) * 10 for j in range(4))
        print(f"frame {l:2d}: assemble {a0:6d}-{a1:6d} ns | solver wait {w:6d} ready {rd:6d} sweep {sw:6d} "
              f"done {dn:6d} ns")
    print(f"backward {(s[0, 250] - t0) * 10} - {(s[0, 251] - t0) * 10} ns")


if __name__ == "__main__" and os.environ.get("GN_TRACE"):
    trace(T=int(os.environ.get("GN_TRACE_T", "3")), variant=int(os.environ.get("GN_VARIANT", "0")))
