"""Interleaved A/B of two builds of the library on one box: per round, one subprocess per
build (PERSEUS_AMD_LIB_AB) times every launch of the B = 64 forward (pa_detector_time_launch,
--reps back-to-back launches between HIP events) and the whole forward; medians per launch.

    python tools/so_ab.py perseus_amd/lib/ab/base.so perseus_amd/lib/libperseus_amd.so --rounds 6
"""
import argparse
import json
import os
import statistics
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def child(precision, batch, reps):
    sys.path.insert(0, ROOT)
    import numpy as np
    import torch

    from perseus_amd import synth
    from perseus_amd.detector import KeypointCNN

    m = KeypointCNN(num_channels=4, precision=precision)
    m.load_state_dict({k: torch.from_numpy(np.asarray(v)) for k, v in synth.synthetic_state_dict(0).items()})
    x = torch.from_numpy(synth.synthetic_frames(0, batch)).cuda()
    m.reserve(batch)
    y = m(x)
    for _ in range(20):
        m(x)
    s = torch.cuda.current_stream()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(s)
    for _ in range(50):
        m(x)
    e1.record(s)
    torch.cuda.synchronize()
    fwd = e0.elapsed_time(e1) / 50 * 1e3
    n = len(m.profile(x)[0])
    per = [m.time_launch(x, i, reps) for i in range(n)]
    y2 = m(x)
    print(json.dumps({"fwd_us": fwd, "launch": [[nm, ms * 1e3] for nm, ms in per],
                      "y": y2.cpu().numpy().ravel()[:64].tolist(), "det": bool(torch.equal(y, y2))}))


def main():
    p = argparse.ArgumentParser()
    p.add_argument("libs", nargs="*")
    p.add_argument("--rounds", type=int, default=6)
    p.add_argument("--precision", default="fp16")
    p.add_argument("--batch", type=int, default=64)
    p.add_argument("--reps", type=int, default=10)
    p.add_argument("--child", action="store_true")
    a = p.parse_args()
    if a.child:
        return child(a.precision, a.batch, a.reps)
    res = {lib: [] for lib in a.libs}
    for r in range(a.rounds):
        for lib in a.libs:
            env = dict(os.environ, PERSEUS_AMD_LIB_AB=os.path.abspath(lib))
            out = subprocess.run([sys.executable, os.path.abspath(__file__), "--child", "--precision", a.precision,
                                  "--batch", str(a.batch), "--reps", str(a.reps)], env=env, capture_output=True,
                                 text=True, timeout=300)
            if out.returncode != 0:
                print(out.stdout[-2000:], out.stderr[-4000:])
                raise SystemExit(f"child failed for {lib}")
            res[lib].append(json.loads(out.stdout.strip().splitlines()[-1]))
            print(f"round {r} {os.path.basename(lib)}: forward {res[lib][-1]['fwd_us']:.1f} us", flush=True)
    base = res[a.libs[0]]
    names = [nm for nm, _ in base[0]["launch"]]
    import numpy as np

    y0 = np.array(base[0]["y"])
    for lib in a.libs[1:]:
        d = np.abs(np.array(res[lib][0]["y"]) - y0).max() * 127.5
        print(f"{os.path.basename(lib)}: max px diff vs {os.path.basename(a.libs[0])} (first 4 frames) = {d:.3e}")
    for i, nm in enumerate(names):
        line = f"{i:02d} {nm:22s}"
        for lib in a.libs:
            line += f" | {os.path.basename(lib)[:12]:12s} {statistics.median(r['launch'][i][1] for r in res[lib]):6.2f}"
        print(line)
    line = "sum of launch medians   "
    for lib in a.libs:
        line += f" | {os.path.basename(lib)[:12]:12s} {sum(statistics.median(r['launch'][i][1] for r in res[lib]) for i in range(len(names))):6.1f}"
    print(line)
    line = "forward (50 back to back)"
    for lib in a.libs:
        line += f" | {os.path.basename(lib)[:12]:12s} {statistics.median(r['fwd_us'] for r in res[lib]):6.1f}"
    print(line)


if __name__ == "__main__":
    main()
