"""Minimal profiling driver: W warm-up + N plain KeypointCNN forwards (no timing
passes), so every run of 18 library dispatches in the trace is one forward in
launch order.  Writes <out>/names.json (launch names, batch) for rocprof_summary.py.

    rocprofv3 --kernel-trace -d DIR -o fwd -- python3 tools/pmc_forward.py --out DIR
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--batch", type=int, default=64)
    p.add_argument("--iters", type=int, default=5)
    p.add_argument("--warmup", type=int, default=2)
    p.add_argument("--precision", default="fp16")
    p.add_argument("--out", required=True)
    p.add_argument("--variant", action="append", default=[], help="LAYER:VARIANT (pa_detector_debug_set_variant)")
    a = p.parse_args()
    import numpy as np
    import torch

    from perseus_amd import _lib, synth
    from perseus_amd.detector import KeypointCNN

    dev = torch.device("cuda", 0)
    m = KeypointCNN(num_channels=4, precision=a.precision)
    m.load_state_dict({k: torch.from_numpy(np.asarray(v)) for k, v in synth.synthetic_state_dict(0).items()})
    m.set_variants(dict(tuple(int(t) for t in lv.split(":")) for lv in a.variant))
    x = torch.from_numpy(synth.synthetic_frames(0, a.batch)).to(dev)
    m.reserve(a.batch, dev)
    with torch.no_grad():
        for _ in range(a.warmup + a.iters):
            m(x)
    torch.cuda.synchronize()
    # launch names come from the library's own profile pass (the last forward in the trace)
    names = [n for n, _ in m.profile(x)[0]]
    torch.cuda.synchronize()
    os.makedirs(a.out, exist_ok=True)
    with open(os.path.join(a.out, "names.json"), "w") as fh:
        from bench import csrc_digest

        json.dump({"batch": a.batch, "precision": a.precision, "names": names, "csrc": csrc_digest(),
                   "forwards": a.warmup + a.iters + 1}, fh)
    print(f"{a.warmup + a.iters + 1} forwards x {len(names)} launches, B={a.batch}")


if __name__ == "__main__":
    main()
