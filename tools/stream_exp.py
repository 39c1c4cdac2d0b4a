"""Throughput experiment: one B=64 forward per step on one stream vs. the same frames split
over two streams (two detector handles), and a hipGraph replay of the B=64 forward.
Prints one JSON line per variant (frames/s over `--steps` steps after `--warmup`)."""

from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from perseus_amd import synth  # noqa: E402
from perseus_amd.detector import KeypointCNN  # noqa: E402


def make(state, dev, B):
    m = KeypointCNN(num_channels=4, precision="fp16")
    m.load_state_dict({k: torch.from_numpy(np.asarray(v)) for k, v in state.items()})
    m.eval()
    m.reserve(B, dev)
    return m


def timed(fn, steps, warmup):
    for _ in range(warmup):
        fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        fn()
    torch.cuda.synchronize()
    return time.perf_counter() - t0


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=20)
    a = ap.parse_args()
    dev = torch.device("cuda:0")
    state = synth.synthetic_state_dict(0)
    x64 = torch.from_numpy(synth.synthetic_frames(0, 64)).to(dev)
    out = []
    with torch.no_grad():
        m0 = make(state, dev, 64)
        t = timed(lambda: m0(x64), a.steps, a.warmup)
        out.append(("1x64", 64 * a.steps / t))
        for split in (32, 64):
            ma, mb = make(state, dev, split), make(state, dev, split)
            xa, xb = x64[:split], x64[64 - split:]
            sa, sb = torch.cuda.Stream(), torch.cuda.Stream()

            def two():
                cur = torch.cuda.current_stream()
                sa.wait_stream(cur)
                sb.wait_stream(cur)
                with torch.cuda.stream(sa):
                    ma(xa)
                with torch.cuda.stream(sb):
                    mb(xb)
                cur.wait_stream(sa)
                cur.wait_stream(sb)

            t = timed(two, a.steps, a.warmup)
            out.append((f"2x{split}", 2 * split * a.steps / t))
        try:
            s = torch.cuda.Stream()
            s.wait_stream(torch.cuda.current_stream())
            with torch.cuda.stream(s):
                m0(x64)
            torch.cuda.current_stream().wait_stream(s)
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g):
                m0(x64)
            t = timed(g.replay, a.steps, a.warmup)
            out.append(("graph1x64", 64 * a.steps / t))
        except Exception as e:  # noqa: BLE001
            out.append(("graph1x64", repr(e)[:200]))
    for k, v in out:
        print(json.dumps({"variant": k, "frames_per_s": v}), flush=True)


if __name__ == "__main__":
    main()
