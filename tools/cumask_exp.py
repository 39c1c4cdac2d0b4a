"""CU-partitioned half-batches: the B = 64 forward as two B = 32 forwards on two HIP streams whose
CU masks (hipExtStreamCreateWithCUMask) split every XCD in half, against the one-stream B = 64
forward, interleaved rounds in one process.  The halves run the same kernels on disjoint CUs, so
their launch-edge bursts (prologue loads, store drains, boundaries) fall at different times
instead of all 256 CUs bursting together.

    python tools/cumask_exp.py [--steps 200] [--rounds 5]
"""
import argparse
import ctypes as C
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def masked_stream(hip, words):
    s = C.c_void_p()
    arr = (C.c_uint32 * len(words))(*words)
    rc = hip.hipExtStreamCreateWithCUMask(C.byref(s), len(words), arr)
    assert rc == 0, f"hipExtStreamCreateWithCUMask: {rc}"
    return s


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--steps", type=int, default=200)
    p.add_argument("--rounds", type=int, default=5)
    a = p.parse_args()
    import numpy as np
    import torch

    from perseus_amd import synth
    from perseus_amd.detector import KeypointCNN

    hip = C.CDLL("libamdhip64.so")
    dev = torch.device("cuda", 0)
    ncu = torch.cuda.get_device_properties(dev).multi_processor_count
    nw = (ncu + 31) // 32
    masks = {
        "alt_bits": ([0x55555555] * nw, [0xAAAAAAAA] * nw),
        "half_words": ([0x0000FFFF] * nw, [0xFFFF0000] * nw),
        "alt_words": ([0xFFFFFFFF if i % 2 == 0 else 0 for i in range(nw)],
                      [0xFFFFFFFF if i % 2 == 1 else 0 for i in range(nw)]),
    }
    sd = {k: torch.from_numpy(np.asarray(v)) for k, v in synth.synthetic_state_dict(0).items()}
    x = torch.from_numpy(synth.synthetic_frames(0, 64)).to(dev)
    m0 = KeypointCNN(num_channels=4).eval()
    m0.load_state_dict(sd)
    mA = KeypointCNN(num_channels=4).eval()
    mA.load_state_dict(sd)
    mB = KeypointCNN(num_channels=4).eval()
    mB.load_state_dict(sd)
    y0 = torch.empty((64, 16), device=dev)
    yA = torch.empty((32, 16), device=dev)
    yB = torch.empty((32, 16), device=dev)
    ref = m0(x, out=y0).clone()
    streams = {}
    for name, (wa, wb) in masks.items():
        sa, sb = masked_stream(hip, wa), masked_stream(hip, wb)
        streams[name] = (torch.cuda.ExternalStream(sa.value, device=dev), torch.cuda.ExternalStream(sb.value, device=dev))
    main_s = torch.cuda.current_stream(dev)

    def one_stream(n):
        for _ in range(n):
            m0(x, out=y0)

    def split(n, sa, sb):
        ea = torch.cuda.Event()
        ea.record(main_s)
        sa.wait_event(ea)
        sb.wait_event(ea)
        for _ in range(n):
            with torch.cuda.stream(sa):
                mA(x[:32], out=yA)
            with torch.cuda.stream(sb):
                mB(x[32:], out=yB)
        fa, fb = torch.cuda.Event(), torch.cuda.Event()
        fa.record(sa)
        fb.record(sb)
        main_s.wait_event(fa)
        main_s.wait_event(fb)

    for name, (sa, sb) in streams.items():
        split(3, sa, sb)
        torch.cuda.synchronize()
        ok = torch.equal(torch.cat((yA, yB)), ref)
        print(f"{name}: halves bit-identical to the B = 64 forward: {ok}", flush=True)
    res = {k: [] for k in ["one_stream"] + list(streams)}
    import time
    for r in range(a.rounds + 1):
        for k in res:
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            if k == "one_stream":
                one_stream(a.steps)
            else:
                split(a.steps, *streams[k])
            torch.cuda.synchronize()
            dt = time.perf_counter() - t0
            if r > 0:
                res[k].append(64 * a.steps / dt)
    for k, v in res.items():
        print(f"{k:12s} median {statistics.median(v) / 1e3:7.1f}k frames/s  (min {min(v) / 1e3:.1f}k, max {max(v) / 1e3:.1f}k)",
              flush=True)


if __name__ == "__main__":
    main()
