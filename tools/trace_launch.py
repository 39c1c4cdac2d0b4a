"""Per-workgroup phase timeline of one forward launch from a timestamping kernel
variant (pa_detector_debug_set_trace; conv.h trace_stamp, s_memrealtime = 100 MHz).

    python tools/trace_launch.py --layer 1 --variant 36 --launch 1 2 3 4

For each traced launch prints, per stamp slot, the median / min / max over
workgroups of (stamp - earliest slot-0 stamp) in us.
"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--layer", type=int, nargs="+", required=True)
    p.add_argument("--variant", type=int, required=True)
    p.add_argument("--launch", type=int, nargs="+", required=True)
    p.add_argument("--batch", type=int, default=64)
    p.add_argument("--runs", type=int, default=5)
    p.add_argument("--precision", default="fp16")
    a = p.parse_args()
    import numpy as np
    import torch

    from perseus_amd import _lib, synth
    from perseus_amd.detector import KeypointCNN

    L = _lib.lib()
    m = KeypointCNN(num_channels=4, precision=a.precision)
    m.load_state_dict({k: torch.from_numpy(np.asarray(v)) for k, v in synth.synthetic_state_dict(0).items()})
    x = torch.from_numpy(synth.synthetic_frames(0, a.batch)).cuda()
    buf = torch.zeros(24 * 65536, dtype=torch.int64, device="cuda")
    m.set_variants({layer: a.variant for layer in a.layer})
    m.set_trace(buf)
    for _ in range(a.runs):
        buf.zero_()
        m(x)
        torch.cuda.synchronize()
    m.set_trace(None)
    m.set_variants({})
    t = buf.view(24, -1, 64).cpu().numpy()
    for li in a.launch:
        tl = t[li]
        wg = np.nonzero(tl[:, 0])[0]
        if len(wg) == 0:
            print(f"launch {li}: no stamps")
            continue
        tl = tl[wg]
        t0 = tl[:, 0].min()
        print(f"launch {li}: {len(wg)} workgroups; end-of-kernel max {(tl[:, 63].max() - t0) / 100:.2f} us")
        if tl[:, 63].any():  # end time by dispatch half (which workgroups win arbitration)
            h = len(wg) // 2
            e = (tl[:, 63] - t0) / 100.0
            print(f"  end by half: first {np.median(e[:h]):.2f} (max {e[:h].max():.2f})  "
                  f"second {np.median(e[h:]):.2f} (max {e[h:].max():.2f}); by parity: even {np.median(e[0::2]):.2f} "
                  f"odd {np.median(e[1::2]):.2f}")
        for s in range(64):
            col = tl[:, s]
            if not col.any():
                continue
            d = (col - t0) / 100.0
            print(f"  slot {s:2d}: median {np.median(d):6.2f}  min {d.min():6.2f}  max {d.max():6.2f}")


if __name__ == "__main__":
    main()
