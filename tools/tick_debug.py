"""Debug: the fused pose tick's two kernels one at a time (pa_debug_gn_set_assemblers 1024:
linearize kernel only, 2048: GN kernel only), each synchronised, progress printed."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import numpy as np
    import torch

    from perseus_amd import _lib, pipeline, synth

    L_ = _lib.lib()
    dev = torch.device("cuda", 0)
    T, L = 3, 6
    tr = synth.synthetic_trajectories(1, T, L)
    y = torch.as_tensor(tr["y"], device=dev)
    a, lin = pipeline.prepare_trajectories(y, tr["poses"], tr["vels"], tr["angvels"], tr["corners"], tr["K"], T=T, L=L,
                                           dt=1 / 30, proj_sigmas=[2.0, 2.0], dyn_sigmas=[0.1] * 6,
                                           cv_sigmas=[0.5] * 3, nvalid=torch.full((T,), int(os.environ.get("TICK_NV", L)),
                                                                                  dtype=torch.int32, device=dev))
    print("prepared", flush=True)
    y_new = torch.as_tensor(tr["y"][:T], device=dev).contiguous()
    delta = torch.zeros((T * L, 12), dtype=torch.float64, device=dev)
    info = torch.zeros(T, dtype=torch.int32, device=dev)
    newest = torch.zeros((T, 12), dtype=torch.float64, device=dev)
    seq = os.environ.get("TICK_SEQ", "0,s,1024,s,2048,s,1024,2048,s").split(",")
    for v in seq:
        if v == "s":
            torch.cuda.synchronize()
            print("sync ok", info.tolist(), float(delta.abs().max()), flush=True)
            continue
        _lib.check(L_.pa_debug_gn_set_assemblers(int(v)))
        pipeline.window_pose_tick(a, y_new, lam=1e-2, delta=delta, info=info, newest=newest)
        print("launched", v, flush=True)
    _lib.check(L_.pa_debug_gn_set_assemblers(0))


main()
