"""ORACLE-side analysis (test infrastructure, CPU only): where the fp16 path's keypoint
error comes from, layer by layer ("next" item 4).

    python oracle/error_attribution.py [--frames 8] [--out profiles/r03_error_attribution.json]

The fp16 product path (perseus_amd) computes every conv as
fp16(BN-folded weight) x fp16(stored activation), accumulated in f32, plus an f32 bias;
activations are stored in fp16 between launches, the residual is added from its fp16
copy.  Relative to the exact forward (f64 here, `resnet_ref.forward`'s graph,
perseus/detector/models.py:34-40 over torchvision's ResNet-18 with eval BatchNorm) its
error sources per conv i are:
  * W_i  rounding the folded weights of conv i to fp16;
  * X_i  rounding conv i's input activation to fp16 (the stored map it reads; for the
         stem the f32 frames it converts; conv1 and the downsample of a block entry
         read the same map);
  * R_b  rounding the residual (identity) input of block b to fp16.
Each source is switched on alone in an otherwise exact f64 forward; the script
reports the per-keypoint px-L2 error (px = 127.5 x normalized, validate.py:144-153)
against the exact forward, every source's share of the sum of single-source mean
errors, the conv's share of the network's FLOPs, and the error with ALL sources on
(the fp16 path itself, cross-checked against the GPU's measured 0.047 px max).  A
mixed fp16 / fp16x3 mode pays off only if the error concentrates in layers holding
few FLOPs (the decision rule is written into the output).
"""

from __future__ import annotations

import argparse
import json
import os
import sys

import numpy as np
import torch
import torch.nn.functional as F

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

BN_EPS = 1e-5


def convs(state):
    """The 20 convs in launch order with BN folded in f64 (as pa_detector_create folds
    them): (name, w, b, stride, pad, input key, role)."""
    sd = {k: torch.from_numpy(np.asarray(v)).double() for k, v in state.items()
          if not k.endswith("num_batches_tracked")}

    def fold(wk, bn):
        g, b, m, v = (sd[f"{bn}.{a}"] for a in ("weight", "bias", "running_mean", "running_var"))
        s = g / torch.sqrt(v + BN_EPS)
        return sd[wk] * s[:, None, None, None], b - m * s

    out = []
    w, b = fold("resnet.conv1.weight", "resnet.bn1")
    out.append(("stem", w, b, 2, 3))
    for li in range(1, 5):
        for bi in range(2):
            p = f"resnet.layer{li}.{bi}"
            st = 2 if (li > 1 and bi == 0) else 1
            w, b = fold(p + ".conv1.weight", p + ".bn1")
            out.append((f"l{li}.{bi}.conv1", w, b, st, 1))
            if p + ".downsample.0.weight" in sd:
                w, b = fold(p + ".downsample.0.weight", p + ".downsample.1")
                out.append((f"l{li}.{bi}.ds", w, b, st, 0))
            w, b = fold(p + ".conv2.weight", p + ".bn2")
            out.append((f"l{li}.{bi}.conv2", w, b, 1, 1))
    fc = (sd["resnet.fc.weight"], sd["resnet.fc.bias"])
    return out, fc


def q16(t):
    return t.to(torch.float16).double()


def forward(cv, fc, x, rw=(), rx=(), rr=()):
    """f64 forward over the folded convs; names in rw / rx round that conv's weights /
    input to fp16, block names in rr round that block's residual input."""
    by = {c[0]: c for c in cv}

    def conv(name, h):
        _, w, b, st, pd = by[name]
        if name in rw:
            w = q16(w)
        if name in rx:
            h = q16(h)
        return F.conv2d(h, w, b, stride=st, padding=pd)

    h = F.relu(conv("stem", x))
    h = F.max_pool2d(h, 3, 2, 1)
    for li in range(1, 5):
        for bi in range(2):
            p = f"l{li}.{bi}"
            o = F.relu(conv(p + ".conv1", h))
            o = conv(p + ".conv2", o)
            idn = conv(p + ".ds", h) if (p + ".ds") in by else h
            if p in rr:
                idn = q16(idn)
            h = F.relu(o + idn)
    h = torch.flatten(F.adaptive_avg_pool2d(h, (1, 1)), 1)
    return F.linear(h, fc[0], fc[1])


def px_err(y, y0):
    d = ((y - y0) * 127.5).reshape(y.shape[0], -1, 2)
    l2 = torch.sqrt((d ** 2).sum(-1))
    return float(l2.max()), float(l2.mean())


def out_hw(cv):
    hw, res = 64, {}
    for name, w, _, st, pd in cv:
        if name == "stem":
            res[name] = 128
            continue
        if name.endswith("conv1") or name.endswith("ds"):
            ho = hw // st
            res[name] = ho
        else:
            res[name] = ho
            hw = ho
    return res


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--frames", type=int, default=8)
    p.add_argument("--seed", type=int, default=0)
    p.add_argument("--out", default=os.path.join(ROOT, "profiles", "r03_error_attribution.json"))
    a = p.parse_args()
    from perseus_amd import synth

    torch.set_num_threads(max(1, len(os.sched_getaffinity(0))))
    state = synth.synthetic_state_dict(a.seed)
    x = torch.from_numpy(synth.synthetic_frames(a.seed, a.frames)).double()
    cv, fc = convs(state)
    names = [c[0] for c in cv]
    ohw = out_hw(cv)
    fl = {n: 2.0 * ohw[n] ** 2 * w.shape[0] * w.shape[1] * w.shape[2] * w.shape[3] for n, w, *_ in cv}
    total_fl = sum(fl.values())
    blocks = [f"l{li}.{bi}" for li in range(1, 5) for bi in range(2)]
    with torch.no_grad():
        y0 = forward(cv, fc, x)
        rows = []
        for n in names:
            ew = px_err(forward(cv, fc, x, rw={n}), y0)
            ex = px_err(forward(cv, fc, x, rx={n}), y0)
            eb = px_err(forward(cv, fc, x, rw={n}, rx={n}), y0)
            rows.append({"conv": n, "flop_share": fl[n] / total_fl, "w_max": ew[0], "w_mean": ew[1],
                         "x_max": ex[0], "x_mean": ex[1], "both_max": eb[0], "both_mean": eb[1]})
            print(f"{n:12s} flops {fl[n] / total_fl:6.3f}  W {ew[1]:.2e} ({ew[0]:.2e})  X {ex[1]:.2e} ({ex[0]:.2e})  "
                  f"W+X {eb[1]:.2e} ({eb[0]:.2e})", flush=True)
        res_rows = []
        for b in blocks:
            er = px_err(forward(cv, fc, x, rr={b}), y0)
            res_rows.append({"block": b, "max": er[0], "mean": er[1]})
            print(f"residual {b:6s} {er[1]:.2e} ({er[0]:.2e})", flush=True)
        allq = px_err(forward(cv, fc, x, rw=set(names), rx=set(names), rr=set(blocks)), y0)
        # two-product schemes: x_hi (w_hi + w_lo) keeps only the activation rounding, (x_hi + x_lo) w_hi
        # only the weight rounding
        act_only = px_err(forward(cv, fc, x, rx=set(names), rr=set(blocks)), y0)
        w_only = px_err(forward(cv, fc, x, rw=set(names)), y0)
    print(f"all sources (the fp16 path): max {allq[0]:.4f} px, mean {allq[1]:.4f} px")
    print(f"fp16 activations + exact weights (2-product x_hi(w_hi + w_lo)): max {act_only[0]:.4f} px")
    print(f"fp16 weights + exact activations (2-product (x_hi + x_lo) w_hi): max {w_only[0]:.4f} px")
    tot = sum(r["both_mean"] for r in rows) + sum(r["mean"] for r in res_rows)
    for r in rows:
        r["err_share"] = r["both_mean"] / tot
    for r in res_rows:
        r["err_share"] = r["mean"] / tot
    # decision rule: the smallest FLOP share that holds >= 95 % of
    # the error, taking convs in descending order of error per FLOP
    order = sorted(rows, key=lambda r: -r["err_share"] / r["flop_share"])
    cum_e = sum(r["err_share"] for r in res_rows)  # residual rounding stays with any mode choice
    cum_f, chosen = 0.0, []
    for r in order:
        if cum_e >= 0.95:
            break
        cum_e += r["err_share"]
        cum_f += r["flop_share"]
        chosen.append(r["conv"])
    concentrated = cum_f <= 0.5
    verdict = (f"95 % of the summed single-source error needs convs holding {cum_f:.1%} of the FLOPs "
               f"({len(chosen)} of {len(rows)} convs): " +
               ("concentrated -> a mixed fp16 / fp16x3 mode is worth building" if concentrated else
                "NOT concentrated -> the parity-grade ceiling is the fp16 rate / 3 (every conv needs the "
                "3-product scheme)"))
    print(verdict)
    out = {"frames": a.frames, "seed": a.seed, "all_sources_px": {"max": allq[0], "mean": allq[1]},
           "two_product_schemes_px": {"activations_fp16_weights_split": {"max": act_only[0], "mean": act_only[1]},
                                      "weights_fp16_activations_split": {"max": w_only[0], "mean": w_only[1]}},
           "convs": rows, "residuals": res_rows, "error_share_order": [r["conv"] for r in order],
           "convs_for_95pct": chosen, "flop_share_for_95pct": cum_f, "concentrated": concentrated,
           "verdict": verdict,
           "method": "f64 forward with one fp16 rounding source on at a time (oracle/error_attribution.py)"}
    os.makedirs(os.path.dirname(a.out), exist_ok=True)
    with open(a.out, "w") as fh:
        json.dump(out, fh, indent=1)


if __name__ == "__main__":
    main()
