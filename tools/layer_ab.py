"""Interleaved A/B timing of kernel variants in ONE process (guide rule 24).

    python tools/layer_ab.py --variants 0 1 2 --rounds 10 [--layers 1 2 3 4]

Each round times every launch of the forward per variant (pa_detector_time_launch:
--reps back-to-back launches between two HIP events), variants interleaved; prints
the median and min per (launch, variant).  Outputs are checked against variant 0's
(plain forward) before timing.
"""
import argparse
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--variants", type=int, nargs="+", default=[0, 1])
    p.add_argument("--layers", type=int, nargs="+", default=[0, 1, 2, 3, 4])
    p.add_argument("--rounds", type=int, default=10)
    p.add_argument("--batch", type=int, default=64)
    p.add_argument("--precision", default="fp16")
    p.add_argument("--reps", type=int, default=10)
    p.add_argument("--split-k", type=int, default=0, help="latency mode max batch (pa_detector_set_split_k)")
    a = p.parse_args()
    import numpy as np
    import torch

    from perseus_amd import _lib, synth
    from perseus_amd.detector import KeypointCNN

    L = _lib.lib()
    m = KeypointCNN(num_channels=4, precision=a.precision)
    m.load_state_dict({k: torch.from_numpy(np.asarray(v)) for k, v in synth.synthetic_state_dict(0).items()})
    if a.split_k:
        m.set_split_k(a.split_k)
    x = torch.from_numpy(synth.synthetic_frames(0, a.batch)).cuda()
    ref = None
    res = {}
    for r in range(a.rounds + 1):
        for v in a.variants:
            m.set_variants({layer: v for layer in a.layers})
            if r == 0:
                y = m(x)
                if ref is None:
                    ref = y
                err = (y - ref).abs().max().item() * 127.5
                print(f"variant {v}: max px diff vs variant {a.variants[0]} = {err:.3e}", flush=True)
                continue  # warm-up round
            n = len(m.profile(x)[0])
            for i in range(n):
                name, ms = m.time_launch(x, i, a.reps)
                res.setdefault(i, {}).setdefault(v, []).append((ms, name))
    tot = {v: 0.0 for v in a.variants}
    for i, d in sorted(res.items()):
        line = f"{i:02d} {d[a.variants[0]][0][1]:20s}"
        for v in a.variants:
            t = [x[0] for x in d[v]]
            med = statistics.median(t)
            tot[v] += med
            line += f" | v{v} {med*1e3:6.1f} ({min(t)*1e3:5.1f})"
        print(line)
    print("total " + " | ".join(f"v{v} {tot[v]*1e3:.1f}us" for v in a.variants))
    m.set_variants({})


if __name__ == "__main__":
    main()
