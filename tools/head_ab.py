"""A/B of whole-forward throughput (B=64, fp16) between kernel variants, interleaved runs
of `--steps` back-to-back forwards.  Usage: head_ab.py [--ab LAYER:VARIANT ...]
(default: 7:3, avgpool + fc fused into layer4's last conv, against the shipped separate head)."""

from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from perseus_amd import _lib, synth  # noqa: E402
from perseus_amd.detector import KeypointCNN  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=300)
    ap.add_argument("--rounds", type=int, default=4)
    ap.add_argument("--ab", nargs="*", default=["7:3"])
    a = ap.parse_args()
    L = _lib.lib()
    dev = torch.device("cuda:0")
    m = KeypointCNN(num_channels=4, precision="fp16")
    m.load_state_dict({k: torch.from_numpy(np.asarray(v)) for k, v in synth.synthetic_state_dict(0).items()})
    m.eval()
    x = torch.from_numpy(synth.synthetic_frames(0, 64)).to(dev)
    m.reserve(64, dev)
    out = torch.empty((64, 16), device=dev)
    variants = [("shipped", [])] + [(s, [tuple(map(int, s.split(":")))]) for s in a.ab]
    res = {k: [] for k, _ in variants}
    with torch.no_grad():
        for _ in range(a.rounds):
            for name, vs in variants:
                m.set_variants(dict(vs))
                for _ in range(20):
                    m(x, out=out)
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                for _ in range(a.steps):
                    m(x, out=out)
                torch.cuda.synchronize()
                res[name].append(64 * a.steps / (time.perf_counter() - t0))
                m.set_variants({})
    for k, v in res.items():
        print(json.dumps({"variant": k, "frames_per_s_median": float(np.median(v)), "runs": [round(u) for u in v]}),
              flush=True)


if __name__ == "__main__":
    main()
