"""Per-pair phase times of the role-split stem (variant 0:24, s_memrealtime stamps per
workgroup, stem.hip stem_role_fp16 DBG = 4): for each conv-row pair, how long the
convolving wave 0 and the row-moving wave 4 worked between barriers, and how long the
barrier held wave 0.  Medians over workgroups, us.

    python3 tools/stem_trace.py
"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import numpy as np
    import torch

    from perseus_amd import synth
    from perseus_amd.detector import KeypointCNN

    m = KeypointCNN(num_channels=4)
    m.load_state_dict({k: torch.from_numpy(np.asarray(v)) for k, v in synth.synthetic_state_dict(0).items()})
    x = torch.from_numpy(synth.synthetic_frames(0, 64)).cuda()
    buf = torch.zeros(24 * 65536, dtype=torch.int64, device="cuda")
    m.set_variants({0: 24})
    m.set_trace(buf)
    for _ in range(5):
        buf.zero_()
        m(x)
        torch.cuda.synchronize()
    t = buf[:256 * 64].cpu().numpy().reshape(256, 64).astype(np.float64) / 100.0  # us, launch 0 (stem)
    t0 = t[:, 60].min()
    med = lambda a: round(float(np.median(a)), 3)
    prev = t[:, 61]
    rows = []
    for j in range(17):
        w0 = t[:, j] - prev          # convolving wave: work of pair j
        w4 = t[:, 20 + j] - prev     # moving wave: work of pair j
        hold = t[:, 40 + j] - t[:, j]  # wave 0 waiting at the barrier
        rows.append({"pair": j, "mfma_wave": med(w0), "mover_wave": med(w4), "wave0_barrier_wait": med(hold)})
        prev = t[:, 40 + j]
    raw = buf[:256 * 64].cpu().numpy().reshape(256, 64).astype(np.float64)
    clk = (raw[:, 59] - raw[:, 58]) / ((raw[:, 62] - raw[:, 60]) / 100.0)  # s_memtime ticks per us
    out = {"shader_clock_ghz": round(float(np.median(clk)) / 1e3, 3), "prologue": med(t[:, 61] - t[:, 60]), "start_skew": med(t[:, 60] - t0),
           "wave0_done": med(t[:, 62] - t0), "wave4_done": med(t[:, 63] - t0), "pairs": rows}
    print(json.dumps(out))


if __name__ == "__main__":
    main()
