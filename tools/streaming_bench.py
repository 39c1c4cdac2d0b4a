"""Config 4: 3 x 720p RGBD cameras at 30 Hz, end-to-end keypoint and pose latency on 1 GPU.

The measurement is bench.py's `streaming_leg` (the same numbers appear in every bench
line as "streaming"): per tick, stage the 3 frames (host -> pinned, centre crop), one
hipGraph replay (H2D, preprocess, B=3 forward, denormalize, D2H; with the pose stage
also window advance, factor linearize, GN step, retract, D2H poses), wait.  Prints one
JSON line.

    python tools/streaming_bench.py [--ticks 300] [--hz 30] [--window 24]
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--ticks", type=int, default=300)
    p.add_argument("--hz", type=float, default=30.0)
    p.add_argument("--cams", type=int, default=3)
    p.add_argument("--window", type=int, default=24)
    p.add_argument("--zero-copy", type=int, default=None, help="1 / 0: the tick reads the pinned staging (no H2D copy); default per precision")
    p.add_argument("--zero-copy-out", type=int, default=1, help="1 / 0: results written into the pinned block (no D2H copy)")
    a = p.parse_args()
    import numpy as np
    import torch

    from bench import streaming_leg
    from perseus_amd import synth
    from perseus_amd.detector import KeypointCNN

    m = KeypointCNN(num_channels=4)
    m.load_state_dict({k: torch.from_numpy(np.asarray(v)) for k, v in synth.synthetic_state_dict(0).items()})
    dev = torch.device("cuda", 0)
    print(json.dumps(streaming_leg(m, dev, a.ticks, a.hz, a.cams, a.window, zero_copy=None if a.zero_copy is None else bool(a.zero_copy),
                                   zero_copy_out=bool(a.zero_copy_out))))


if __name__ == "__main__":
    main()
