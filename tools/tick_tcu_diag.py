"""Diagnostic: the fused pose tick (pa_window_pose_tick) against the four separate launches
(cyclic reduction forced) at several trajectory counts T, one tick on the same windows; prints
per T the trajectories whose delta differs and the largest difference.

    python tools/tick_tcu_diag.py [--T 3 64 256 257]
"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests"))


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--T", type=int, nargs="+", default=[3, 64, 256, 257])
    p.add_argument("--L", type=int, default=24)
    p.add_argument("--seed", type=int, default=31)
    a = p.parse_args()
    import numpy as np
    import torch

    from perseus_amd import _lib, pipeline, synth
    from test_pose_tick_split_gpu import _setup_rows

    L_ = _lib.lib()
    Tmax, L, nk = max(a.T), a.L, 8
    tr = synth.synthetic_trajectories(a.seed, Tmax, L, n_kp=nk)
    rng = np.random.default_rng(5)
    y_all = (tr["y"].reshape(Tmax, L, -1)[:, -1] + 0.01 * rng.standard_normal((Tmax, 2 * nk))).astype(np.float32)
    for T in a.T:
        fa, flin, fout = _setup_rows(tr, 0, T, L, nk)
        qa, qlin, qout = _setup_rows(tr, 0, T, L, nk)
        keep = qlin["_keep"]
        win = {"y": keep[0].view(T, L, 2 * nk), "pose": keep[1].view(T, L, 12), "vel": keep[2].view(T, L, 3),
               "angvel": keep[3].view(T, L, 3)}
        plan = pipeline.GNPlan(qlin, T=T, L=L, lam=1e-2)
        plan.out["delta"], plan.out["info"] = qout["delta"], qout["info"]
        y_new = torch.as_tensor(y_all[:T], device="cuda").contiguous()
        pipeline.window_pose_tick(fa, y_new, lam=1e-2, **fout)
        L_.pa_debug_gn_set_assemblers(64)
        try:
            pipeline.window_advance(y_new, win, dt=1 / 30, nvalid=keep[10])
            pipeline.launch(qa, torch.device("cuda", 0))
            torch.cuda.synchronize()
            lin_eq = {k: torch.equal(v, qlin[k]) for k, v in flin.items() if isinstance(v, torch.Tensor)}
            plan.launch()
            pipeline.window_retract(win, qout["delta"], qout["info"], newest=qout["newest"])
            torch.cuda.synchronize()
        finally:
            L_.pa_debug_gn_set_assemblers(0)
        df = fout["delta"].view(T, -1)
        dq = qout["delta"].view(T, -1)
        bad = (df != dq).any(1).nonzero().flatten().tolist()
        diff = (df - dq).abs().max().item()
        print(f"T={T}: lin equal {all(lin_eq.values())} ({[k for k, v in lin_eq.items() if not v]}); "
              f"delta mismatched trajectories {len(bad)} {bad[:10]} max |diff| {diff:.3e}; info equal "
              f"{torch.equal(fout['info'], qout['info'])}; newest equal {torch.equal(fout['newest'], qout['newest'])}",
              flush=True)


if __name__ == "__main__":
    main()
