"""Latency mode A/B: the fp16 forward of a few frames (the streaming pose stage's batch,
one frame per camera) with the batched kernels against pa_detector_set_split_k
(conv_splitk.hip), each captured in a hipGraph and replayed back to back, interleaved
rounds in one process.  Prints one JSON line per batch size.

    python tools/splitk_ab.py [--batches 1,3,8] [--reps 200] [--rounds 5]
"""
import argparse
import json
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--batches", default="1,3,8")
    p.add_argument("--reps", type=int, default=200)
    p.add_argument("--rounds", type=int, default=5)
    p.add_argument("--variants", default="", help="a third mode: split-K plus these kernel variants, e.g. 2:51,6:12")
    a = p.parse_args()
    extra = {int(k): int(v) for k, v in (kv.split(":") for kv in a.variants.split(",") if kv)}
    import numpy as np
    import torch

    from perseus_amd import synth
    from perseus_amd.detector import KeypointCNN

    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    for B in [int(b) for b in a.batches.split(",")]:
        x = torch.from_numpy(synth.synthetic_frames(0, B)).to(dev)
        graphs = {}
        modes = [("batched", 0, {}), ("split_k", B, {})] + ([("split_k+variants", B, extra)] if extra else [])
        for mode, sk, var in modes:
            m = KeypointCNN(num_channels=4)
            m.load_state_dict({k: torch.from_numpy(np.asarray(v)) for k, v in synth.synthetic_state_dict(0).items()})
            m.set_split_k(sk)
            m.set_variants(var)
            y = torch.empty((B, 16), dtype=torch.float32, device=dev)
            s = torch.cuda.Stream(dev)
            with torch.cuda.stream(s):
                m.reserve(B)
                m(x, out=y)
                torch.cuda.synchronize()
                g = torch.cuda.CUDAGraph()
                with torch.cuda.graph(g, stream=s):
                    m(x, out=y)
            graphs[mode] = (m, g, y)
        t = {k: [] for k in graphs}
        for _ in range(a.rounds):
            for mode, (_, g, _) in graphs.items():
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                g.replay()
                torch.cuda.synchronize()
                e0.record()
                for _ in range(a.reps):
                    g.replay()
                e1.record()
                torch.cuda.synchronize()
                t[mode].append(e0.elapsed_time(e1) * 1e3 / a.reps)
        ya, yb = graphs["batched"][2], graphs["split_k"][2]
        print(json.dumps({"B": B, **{f"{k}_us": round(statistics.median(v), 2) for k, v in t.items()},
                          "rounds": {k: [round(u, 2) for u in v] for k, v in t.items()},
                          "max_px_diff": float((ya - yb).abs().max()) * 127.5}), flush=True)


if __name__ == "__main__":
    main()
