"""zero_copy=True ticks equal the copying ticks bit for bit (pixels, poses, info), fp16 and fp16x3."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import numpy as np
    import torch

    from perseus_amd import synth
    from perseus_amd.detector import KeypointCNN
    from perseus_amd.streaming import StreamingPipeline

    for prec in ("fp16", "fp16x3"):
        m = KeypointCNN(num_channels=4, precision=prec)
        m.load_state_dict({k: torch.from_numpy(np.asarray(v)) for k, v in synth.synthetic_state_dict(0).items()})
        a = StreamingPipeline(m, pose_window=6, proj_sigma=40.0)
        b = StreamingPipeline(m, pose_window=6, proj_sigma=40.0, zero_copy=True)
        rng = np.random.default_rng(3)
        for i in range(8):
            rgb = rng.integers(0, 256, (3, 720, 1280, 3), dtype=np.uint8)
            dep = rng.uniform(0.2, 2.0, (3, 720, 1280)).astype(np.float32)
            ra, rb = a.tick(rgb, dep), b.tick(rgb, dep)
            for x, y in zip(ra, rb):
                np.testing.assert_array_equal(x, y)
        print(prec, "zero-copy ticks bit-identical", flush=True)
        a.close()
        b.close()


main()
