"""Per-launch roofline table (markdown) from a bench JSON line's kernels_ms and the
committed PMC traffic: algorithmic FLOPs and bytes per launch (fp16 NHWC activations,
f32 NCHW stem input, fp16 weights), measured time, MFMA and HBM fractions.

    python tools/roofline_table.py gpurun_out/r01/bench.log
"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from bench import HBM_PEAK, MFMA_FP16_DENSE_PEAK, conv_flops  # noqa: E402


def conv_bytes(B):
    """Algorithmic HBM bytes per launch: every operand once (fp16 = 2 B)."""
    by = [B * 4 * 256 * 256 * 4 + B * 64 * 64 * 64 * 2 + 64 * 4 * 49 * 2]  # stem: f32 in, pooled fp16 out
    hw, cin = 64, 64
    for li, cout in enumerate((64, 128, 256, 512)):
        for bi in range(2):
            s = 2 if (li > 0 and bi == 0) else 1
            ho = hw // s
            c_in = cin if bi == 0 else cout
            act_in = B * hw * hw * c_in * 2
            act_out = B * ho * ho * cout * 2
            w1 = cout * 9 * c_in * 2
            if bi == 0 and li > 0:
                by.append(act_in + 2 * act_out + w1 + cout * c_in * 2)  # conv1 out + downsample out
            else:
                by.append(act_in + act_out + w1)
            by.append(act_out + act_out + act_out + cout * 9 * cout * 2)  # conv2: in, residual, out
            hw = ho
        cin = cout
    by.append(B * 8 * 8 * 512 * 2 + 512 * 16 * 4 + B * 16 * 4)
    return by


def main():
    line = [json.loads(ln) for ln in open(sys.argv[1]) if ln.startswith("{")][-1]
    B = line["config"]["per_gpu_batch"]
    ks = line["kernels_ms"]
    fl = conv_flops(B)
    by = conv_bytes(B)
    tr = None
    tf = os.path.join(ROOT, "profiles", "pmc_traffic.json")
    if os.path.exists(tf):
        tr = json.load(open(tf)).get("fp16", {}).get("bytes_per_launch")
    print("| # | launch | us | GFLOP | MFMA frac | alg. MB | HBM frac (alg.) | PMC MB |")
    print("|---|---|---|---|---|---|---|---|")
    tot_t = tot_f = 0.0
    for i, (k, ms) in enumerate(ks.items()):
        t = ms * 1e-3
        tot_t += t
        tot_f += fl[i]
        pm = f"{tr[i] / 1e6:.1f}" if tr else "-"
        print(f"| {i:02d} | {k[3:]} | {ms * 1e3:.1f} | {fl[i] / 1e9:.2f} | {fl[i] / t / MFMA_FP16_DENSE_PEAK:.3f} | "
              f"{by[i] / 1e6:.1f} | {by[i] / t / HBM_PEAK:.3f} | {pm} |")
    print(f"| | total | {tot_t * 1e6:.0f} | {tot_f / 1e9:.1f} | {tot_f / tot_t / MFMA_FP16_DENSE_PEAK:.3f} | "
          f"{sum(by) / 1e6:.0f} | {sum(by) / tot_t / HBM_PEAK:.3f} | |")


if __name__ == "__main__":
    main()
