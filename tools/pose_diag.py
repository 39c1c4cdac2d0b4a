"""Diagnostic for the pose tick's GN step (tests/test_streaming_pose_gpu.py's window):
per trajectory the GPU info / delta against the dense oracle, the conditioning of
H + lam I, and the same tick with the latency mode off.

    python tools/pose_diag.py
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))


def run(split_k):
    import numpy as np
    import torch

    from oracle import gn_ref as G
    from perseus_amd import synth
    from perseus_amd.detector import KeypointCNN
    from perseus_amd.streaming import StreamingPipeline
    from test_streaming_gpu import _frames
    from test_streaming_pose_gpu import LW, SIG, _init

    m = KeypointCNN(num_channels=4)
    m.load_state_dict({k: torch.from_numpy(np.asarray(v)) for k, v in synth.synthetic_state_dict(0).items()})
    p0, v0, w0 = _init()
    p = StreamingPipeline(m, graph=True, pose_window=LW, init_pose=p0, init_vel=v0, init_angvel=w0, split_k=split_k,
                          **SIG)
    for seed in range(1, LW):
        p.tick(*_frames(seed))
    px, pose, info = p.tick(*_frames(99))
    lin = {k: (v.transpose(1, 2) if k.startswith("j_") else v) for k, v in p.lin.items() if isinstance(v, torch.Tensor)}
    f = {k: lin[k].cpu().numpy() for k in ("r_proj", "j_proj", "status", "r_dyn", "j_dyn0", "j_dyn1", "j_dyn2",
                                           "j_dyn3", "r_cv", "j_cv0", "j_cv1")}
    H, g, d = G.gn_step(f, 3, LW, m.n_keypoints, SIG["lam"])
    dd = p.gn.out["delta"].cpu().numpy().reshape(3, -1)
    print(f"split_k={split_k} info={info.tolist()} status={np.bincount(f['status'].ravel()).tolist()}")
    for t in range(3):
        M = H[t] + SIG["lam"] * np.eye(H.shape[1])
        ev = np.linalg.eigvalsh(M)
        # 2x2 pivot dets of the first frame's block (the sweep's first pivots)
        D0 = M[:12, :12]
        dets = [D0[k, k] * D0[k + 1, k + 1] - D0[k, k + 1] ** 2 for k in range(0, 12, 2)]
        print(f"  t={t} eig min {ev.min():.3e} max {ev.max():.3e} cond {ev.max() / ev.min():.3e} "
              f"|d| {np.abs(d[t]).max():.3e} gpu-nan {np.isnan(dd[t]).sum()} "
              f"max|gpu-d| {np.nanmax(np.abs(dd[t] - d[t])) if not np.isnan(dd[t]).all() else float('nan'):.3e}")
        print(f"      diag(M) min {np.diag(M).min():.3e} max {np.diag(M).max():.3e} frame0 dets {['%.2e' % x for x in dets]}")
    p.close()


if __name__ == "__main__":
    import numpy as np

    np.set_printoptions(linewidth=200)
    run(True)
    run(False)
