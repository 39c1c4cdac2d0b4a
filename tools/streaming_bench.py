"""Config 4: 3 x 720p RGBD cameras at 30 Hz, end-to-end keypoint latency on 1 GPU.

Per tick: stage the 3 frames (host -> pinned, centre crop), one hipGraph replay
(H2D, preprocess, B=3 forward, denormalize, D2H), wait.  Latency = stage start to
pixels on the host.  Ticks are paced at --hz (camera rate); reports p50/p99/max over
--ticks for each mode.  Prints one JSON line.

    python tools/streaming_bench.py [--ticks 300] [--hz 30]
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
    p.add_argument("--ticks", type=int, default=300)
    p.add_argument("--hz", type=float, default=30.0)
    p.add_argument("--cams", type=int, default=3)
    a = p.parse_args()
    import numpy as np
    import torch

    from perseus_amd import synth
    from perseus_amd.detector import KeypointCNN
    from perseus_amd.streaming import StreamingPipeline

    m = KeypointCNN(num_channels=4)
    m.load_state_dict({k: torch.from_numpy(np.asarray(v)) for k, v in synth.synthetic_state_dict(0).items()})
    rng = np.random.default_rng(0)
    n_src = 8  # rotate through a few distinct synthetic camera ticks
    rgbs = rng.integers(0, 256, (n_src, a.cams, 720, 1280, 3), dtype=np.uint8)
    deps = rng.uniform(0.12, 0.48, (n_src, a.cams, 720, 1280)).astype(np.float32)
    res = {}
    for name, kw in (("graph_hostcrop", dict(graph=True, host_crop=True)),
                     ("graph_fullframe", dict(graph=True, host_crop=False)),
                     ("eager_hostcrop", dict(graph=False, host_crop=True))):
        pipe = StreamingPipeline(m, n_cams=a.cams, **kw)
        for i in range(10):
            pipe(rgbs[i % n_src], deps[i % n_src])
        lat = []
        period = 1.0 / a.hz
        t_next = time.perf_counter()
        for i in range(a.ticks):
            while time.perf_counter() < t_next:
                pass
            t0 = time.perf_counter()
            pipe(rgbs[i % n_src], deps[i % n_src])
            lat.append(time.perf_counter() - t0)
            t_next += period
        lat = np.array(lat) * 1e3
        # device-only time of one replay
        s = pipe.stream
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        with torch.cuda.stream(s):
            e0.record(s)
            for _ in range(20):
                if pipe.graph is None:
                    pipe._enqueue()
                else:
                    pipe.graph.replay()
            e1.record(s)
        s.synchronize()
        res[name] = {"p50_ms": round(float(np.percentile(lat, 50)), 4), "p99_ms": round(float(np.percentile(lat, 99)), 4),
                     "max_ms": round(float(lat.max()), 4), "device_ms_per_tick": round(e0.elapsed_time(e1) / 20, 4)}
    print(json.dumps({"workload": f"streaming_{a.cams}x720p_rgbd_{a.hz:g}hz", "ticks": a.ticks, "unit": "ms",
                      "latency": res, "note": "latency = host staging + one tick on the GPU + pixels back on host"}))


if __name__ == "__main__":
    main()
