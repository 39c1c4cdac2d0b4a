"""Profiling driver for the factor path (configs[3] side): pa_trajectory_linearize and
pa_trajectory_gn_step over 1000 trajectories x 24 frames, `--iters` times each, so a
rocprofv3 kernel trace shows every factor kernel's per-launch time.

    rocprofv3 --kernel-trace --stats -d DIR -o fac -- python3 tools/factor_prof.py
"""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--T", type=int, default=1000)
    p.add_argument("--L", type=int, default=24)
    p.add_argument("--iters", type=int, default=10)
    a = p.parse_args()
    import torch

    from perseus_amd import pipeline, synth

    dev = torch.device("cuda", 0)
    tr = synth.synthetic_trajectories(1, a.T, a.L)
    y = torch.as_tensor(tr["y"], device=dev)
    args, out = pipeline.prepare_trajectories(y, tr["poses"], tr["vels"], tr["angvels"], tr["corners"], tr["K"],
                                              T=a.T, L=a.L, dt=1 / 12, proj_sigmas=[1.0, 1.0], dyn_sigmas=[0.1] * 6,
                                              cv_sigmas=[0.1] * 3)
    for _ in range(a.iters):
        pipeline.launch(args, dev)
    for _ in range(a.iters):
        g = pipeline.gn_step(out, T=a.T, L=a.L, lam=1e-3)
    torch.cuda.synchronize()
    print("solved", int((g["info"] == 0).sum()), "of", a.T)


if __name__ == "__main__":
    main()
