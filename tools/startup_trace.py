"""Start-up behaviour of the bench loop (VERDICT r01 "20- vs 200-step gap").

Mimics bench.py: model + reserve, W warm-up forwards, synchronize, then N forwards with
a HIP event between consecutive forwards (device time per forward) and the host time of
each model(x) call.  Prints one line per forward and a summary, so a slow start shows
up as either device time (clocks, first-use state) or host time (Python / ctypes).

    python tools/startup_trace.py [--warmup 5] [--iters 40] [--idle-ms 0]
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--batch", type=int, default=64)
    p.add_argument("--warmup", type=int, default=5)
    p.add_argument("--iters", type=int, default=40)
    p.add_argument("--idle-ms", type=float, default=0.0, help="host sleep between warm-up and timed loop")
    p.add_argument("--precision", default="fp16")
    p.add_argument("--out", default=None)
    a = p.parse_args()
    import numpy as np
    import torch

    from perseus_amd import synth
    from perseus_amd.detector import KeypointCNN

    dev = torch.device("cuda", 0)
    m = KeypointCNN(num_channels=4, precision=a.precision)
    m.load_state_dict({k: torch.from_numpy(np.asarray(v)) for k, v in synth.synthetic_state_dict(0).items()})
    m.eval()
    x = torch.from_numpy(synth.synthetic_frames(0, a.batch)).to(dev)
    m.reserve(a.batch, dev)
    kp = torch.empty((a.iters, a.batch, 16), dtype=torch.float32, device=dev)
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(a.iters + 1)]
    res = {}
    for phase in ("cold", "hot"):
        with torch.no_grad():
            for _ in range(a.warmup):
                m(x)
            torch.cuda.synchronize(dev)
            if a.idle_ms > 0:
                time.sleep(a.idle_ms * 1e-3)
            host = []
            t0 = time.perf_counter()
            ev[0].record()
            for i in range(a.iters):
                h0 = time.perf_counter()
                m(x, out=kp[i])
                host.append((time.perf_counter() - h0) * 1e6)
                ev[i + 1].record()
            t_issue = time.perf_counter() - t0
            torch.cuda.synchronize(dev)
            wall = time.perf_counter() - t0
        dev_us = [ev[i].elapsed_time(ev[i + 1]) * 1e3 for i in range(a.iters)]
        res[phase] = {"device_us": [round(v, 1) for v in dev_us], "host_us": [round(v, 1) for v in host],
                      "issue_ms": round(t_issue * 1e3, 3), "wall_ms": round(wall * 1e3, 3),
                      "first10_dev_us": round(sum(dev_us[:10]) / 10, 1),
                      "last10_dev_us": round(sum(dev_us[-10:]) / 10, 1),
                      "mean_host_us": round(sum(host) / len(host), 1)}
        print(phase, {k: v for k, v in res[phase].items() if not k.endswith("_us") or "10" in k or "mean" in k})
        for i in range(a.iters):
            print(f"  {phase} {i:3d} dev {dev_us[i]:8.1f} us  host {host[i]:7.1f} us")
        # "hot": repeat after a long back-to-back run
        with torch.no_grad():
            for _ in range(500):
                m(x)
    if a.out:
        os.makedirs(a.out, exist_ok=True)
        with open(os.path.join(a.out, "startup.json"), "w") as fh:
            json.dump(res, fh)


if __name__ == "__main__":
    main()
