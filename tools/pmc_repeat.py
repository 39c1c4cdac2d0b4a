"""PMC driver for cache-state comparisons: one plain forward (every launch once, caches as
in the forward), then launch `--launch` of that forward repeated `--reps` times back to back
(pa_detector_time_launch: instruction and data caches warm from the previous rep).

    rocprofv3 --pmc <counters> -d DIR -o p -- python3 tools/pmc_repeat.py --launch 10
"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--launch", type=int, default=10)
    p.add_argument("--reps", type=int, default=5)
    p.add_argument("--batch", type=int, default=64)
    a = p.parse_args()
    import numpy as np
    import torch

    from perseus_amd import synth
    from perseus_amd.detector import KeypointCNN

    m = KeypointCNN(num_channels=4)
    m.load_state_dict({k: torch.from_numpy(np.asarray(v)) for k, v in synth.synthetic_state_dict(0).items()})
    x = torch.from_numpy(synth.synthetic_frames(0, a.batch)).cuda()
    with torch.no_grad():
        m(x)
        m(x)
    torch.cuda.synchronize()
    print(m.time_launch(x, a.launch, a.reps))


if __name__ == "__main__":
    main()
