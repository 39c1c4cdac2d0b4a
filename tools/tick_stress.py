"""Debug: pa_window_pose_tick (or one of its two kernels: TICK_V = 1024 linearize only,
2048 GN only; TICK_SPLIT=1: pa_window_pose_tick_pre + _post, TICK_L the window) N times in a
row, a synchronize every 50, progress printed."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import torch

    from perseus_amd import _lib, pipeline, synth

    L_ = _lib.lib()
    dev = torch.device("cuda", 0)
    T, L = 3, int(os.environ.get("TICK_L", "6"))
    tr = synth.synthetic_trajectories(1, T, L)
    nvalid = torch.zeros((T,), dtype=torch.int32, device=dev)
    y = torch.as_tensor(tr["y"], device=dev)
    a, lin = pipeline.prepare_trajectories(y, tr["poses"], tr["vels"], tr["angvels"], tr["corners"], tr["K"], T=T, L=L,
                                           dt=1 / 30, proj_sigmas=[2.0, 2.0], dyn_sigmas=[0.1] * 6,
                                           cv_sigmas=[0.5] * 3, nvalid=nvalid)
    y_new = torch.as_tensor(tr["y"][:T], device=dev).contiguous()
    delta = torch.zeros((T * L, 12), dtype=torch.float64, device=dev)
    info = torch.zeros(T, dtype=torch.int32, device=dev)
    newest = torch.zeros((T, 12), dtype=torch.float64, device=dev)
    _lib.check(L_.pa_debug_gn_set_assemblers(int(os.environ.get("TICK_V", "0"))))
    n = int(os.environ.get("TICK_N", "1000"))
    split = os.environ.get("TICK_SPLIT", "0") == "1"
    ws = pipeline.window_pose_tick_workspace(T, L, dev)
    for i in range(n):
        if split:
            pipeline.window_pose_tick_pre(a, ws, lam=1e-2)
            pipeline.window_pose_tick_post(a, y_new, ws, delta=delta, info=info, newest=newest)
        else:
            pipeline.window_pose_tick(a, y_new, lam=1e-2, delta=delta, info=info, newest=newest)
        if i % 50 == 49:
            torch.cuda.synchronize()
            print(i + 1, "ok", flush=True)
    _lib.check(L_.pa_debug_gn_set_assemblers(0))


main()
