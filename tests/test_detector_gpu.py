"""GPU parity of the HIP detector (through the C ABI) against the oracle / golden vectors.

Tolerances (north_star: 1e-3 px on keypoint coordinates; px = 127.5 x normalized):
  * fp32 parity mode (exact-f32 MFMA, f32 NHWC) and fp16x3 (the fast parity mode: hi/lo
    fp16 planes, 3 fp16 MFMA products per MAC): max |dpx| <= 1e-3 px vs the reference's
    own f32 CPU outputs (golden) and vs the f64 oracle.
  * fp16 mode (the fast path): measured error reported; bound FP16_PX_MAX below.
"""
import json
import os

import numpy as np
import pytest
import torch

from oracle import resnet_ref as R
from perseus_amd import synth
from perseus_amd.detector import KeypointCNN, denormalize_pixel_coordinates

pytestmark = pytest.mark.gpu
GOLD = os.path.join(os.path.dirname(__file__), "golden")
PX = 127.5
FP32_PX_MAX = 1e-3
# fp16 mode (the headline path) is not a parity mode: a regression bound near what it delivers
# (max observed 0.0848 px on the golden case synthetic_b3_seed7, 0.0548 px over the bench's 64
# frames x 8 keypoints, BENCH_r05; fp16 activations and weights over 20 layers), not the
# north_star's 1e-3 px (was 0.1)
FP16_PX_MAX = 0.09
# fp16 integer pixels (streaming.py:143-144) on the bench batch: mismatches among coordinates
# > 1e-3 px from an integer boundary, at most what round 5 measured (12 of 1,023, BENCH_r05)
FP16_SAFE_INT_MISMATCH_MAX = 12


def model(seed=0, in_ch=4, precision="fp16"):
    m = KeypointCNN(num_channels=in_ch, precision=precision)
    m.load_state_dict({k: torch.from_numpy(np.asarray(v)) for k, v in synth.synthetic_state_dict(seed, in_ch).items()})
    return m.eval()


@pytest.fixture(scope="module")
def gold():
    return dict(np.load(os.path.join(GOLD, "detector_golden.npz")))


def cases():
    from oracle.gen_golden import detector_cases

    return detector_cases()


PARITY_MODES = ("fp32", "fp16x3")


@pytest.mark.parametrize("precision", PARITY_MODES)
@pytest.mark.parametrize("idx", range(4))
def test_parity_modes_match_reference_golden(gold, idx, precision):
    name, seed, x = cases()[idx]
    m = model(seed, precision=precision)
    y = m(torch.from_numpy(x).cuda()).cpu().numpy()
    err_ref = np.abs(y - gold[f"{name}/y_ref_f32"]).max() * PX
    err64 = np.abs(y - gold[f"{name}/y_oracle_f64"]).max() * PX
    print(f"{name}: {precision} max px err vs ref {err_ref:.3e} vs f64 {err64:.3e}")
    assert err_ref <= FP32_PX_MAX and err64 <= FP32_PX_MAX


@pytest.mark.parametrize("idx", range(4))
def test_fp16_mode_matches_reference_golden(gold, idx):
    name, seed, x = cases()[idx]
    m = model(seed, precision="fp16")
    y = m(torch.from_numpy(x).cuda()).cpu().numpy()
    d = np.abs(y - gold[f"{name}/y_oracle_f64"]).reshape(y.shape[0], -1, 2) * PX
    l2 = np.sqrt((d ** 2).sum(-1))
    print(f"{name}: fp16 px-L2 max {l2.max():.3e} mean {l2.mean():.3e}")
    assert l2.max() <= FP16_PX_MAX


@pytest.mark.parametrize("B", [1, 5, 64])
@pytest.mark.parametrize("precision", ["fp32", "fp16x3", "fp16"])
def test_batch_sizes_vs_oracle(B, precision):
    x = synth.synthetic_frames(3, B, first=17)
    m = model(0, precision=precision)
    y = m(torch.from_numpy(x).cuda()).cpu().numpy()
    y64 = R.run(synth.synthetic_state_dict(0), x, torch.float64)
    d = np.abs(y - y64).reshape(B, -1, 2) * PX
    l2 = np.sqrt((d ** 2).sum(-1))
    tol = FP32_PX_MAX if precision in PARITY_MODES else FP16_PX_MAX
    print(f"B={B} {precision}: px-L2 max {l2.max():.3e} mean {l2.mean():.3e}")
    assert l2.max() <= tol


def _int_px(y):
    """The integer pixels scripts/streaming.py:142-144 draws: int() of the kornia-
    denormalized coordinates (validate.py:144-153 / streaming.py:129-131, f32)."""
    px = R.denormalize_f32(y)
    return px, np.trunc(px).astype(np.int64)


@pytest.mark.parametrize("precision", PARITY_MODES)
@pytest.mark.parametrize("idx", range(4))
def test_integer_keypoints_parity_modes_bit_exact(gold, idx, precision):
    """north_star: bit-exact integer pixel indices.  The GPU keypoints, denormalized by the
    library's postprocess kernel and truncated as streaming.py:143-144 does, equal the
    reference's own integers for every coordinate farther than the 1e-3 px tolerance from
    an integer boundary (closer ones may legitimately round either way)."""
    name, seed, x = cases()[idx]
    m = model(seed, precision=precision)
    y = m(torch.from_numpy(x).cuda())
    px_gpu = denormalize_pixel_coordinates(y).cpu().numpy()
    px_ref, int_ref = _int_px(gold[f"{name}/y_ref_f32"])
    np.testing.assert_array_equal(px_gpu, R.denormalize_f32(y.cpu().numpy()))
    int_gpu = np.trunc(px_gpu).astype(np.int64)
    safe = np.abs(px_ref - np.round(px_ref)) > FP32_PX_MAX
    assert safe.mean() > 0.9
    bad = int((int_gpu != int_ref)[safe].sum())
    print(f"{name}: {safe.sum()} safe coordinates, {bad} integer mismatches")
    assert bad == 0


@pytest.mark.parametrize("precision", ["fp32", "fp16x3", "fp16"])
def test_integer_keypoints_batch64(precision):
    """Same check on a 64-frame bench batch against the CPU f32 oracle (fp32 mode: zero
    mismatches among safe coordinates; fp16 mode: reported, and bounded by the
    coordinates within FP16_PX_MAX of a boundary)."""
    x = synth.synthetic_frames(0, 64)
    m = model(0, precision=precision)
    y = m(torch.from_numpy(x).cuda()).cpu().numpy()
    px_ref, int_ref = _int_px(R.run(synth.synthetic_state_dict(0), x, torch.float32))
    _, int_gpu = _int_px(y)
    tol = FP32_PX_MAX if precision in PARITY_MODES else FP16_PX_MAX
    frac = np.abs(px_ref - np.round(px_ref))
    mism = int_gpu != int_ref
    safe = frac > FP32_PX_MAX
    print(f"{precision}: {int(mism.sum())} / {mism.size} integer mismatches, {int((mism & safe).sum())} of "
          f"{int(safe.sum())} safe ({int((frac <= tol).sum())} coordinates within {tol} px of a boundary)")
    assert not (mism & (frac > tol)).any()
    if precision == "fp16":
        assert int((mism & safe).sum()) <= FP16_SAFE_INT_MISMATCH_MAX


@pytest.mark.parametrize("precision", PARITY_MODES)
def test_rgb_three_channel_model(precision):
    x = synth.synthetic_frames(1, 2)[:, :3].copy()
    m = model(2, in_ch=3, precision=precision)
    y = m(torch.from_numpy(x).cuda()).cpu().numpy()
    y64 = R.run(synth.synthetic_state_dict(2, 3), x, torch.float64)
    assert np.abs(y - y64).max() * PX <= FP32_PX_MAX


def test_fp16x3_profile_and_precision_switch():
    """fp16x3 runs its own kernels (stem + pool fused, stride-2 + downsample fused) and a
    model switched between modes keeps giving each mode's bits."""
    x = torch.from_numpy(synth.synthetic_frames(0, 8)).cuda()
    m = model(0, precision="fp16x3")
    prof, y = m.profile(x)
    names = [n for n, _ in prof]
    assert names[0] == "stem_x3_conv7x7_pool" and names[-1] == "avgpool_fc_x3" and len(names) == 18
    assert names[5] == "conv3x3s2v3_l2" and names[9] == "conv3x3s2k3_l3" and names[1] == "conv3x3x3_l1"
    assert torch.equal(y, m(x))
    m.precision = "fp16"
    y16 = m(x)
    m.precision = "fp16x3"
    assert torch.equal(m(x), y) and not torch.equal(y16, y)


def test_batch_invariance_and_determinism():
    """Each frame's keypoints are bit-identical whatever batch it is run in (the
    reduction order over K does not depend on the tile shape) and run to run."""
    x = torch.from_numpy(synth.synthetic_frames(5, 64)).cuda()
    for prec in ("fp16", "fp32", "fp16x3"):
        m = model(0, precision=prec)
        y64 = m(x)
        y64b = m(x)
        assert torch.equal(y64, y64b)
        for i in (0, 13, 63):
            y1 = m(x[i:i + 1])
            assert torch.equal(y1[0], y64[i]), (prec, i)


def test_split_k_latency_mode():
    """pa_detector_set_split_k (conv_splitk.hip): batches of up to max_batch frames run the
    stride-1 convs of layers 2-4 as split-K + fixed-order reduce.  Within the fp16 budget of
    the f64 oracle, deterministic, batch-invariant among split-K batches, and larger
    batches keep the batched kernels' bits."""
    xs = synth.synthetic_frames(7, 9, first=3)
    x = torch.from_numpy(xs).cuda()
    m = model(0, precision="fp16")
    y_batched = m(x)
    m.set_split_k(8)
    names = [n for n, _ in m.profile(x[:3])[0]]
    # layers 3 / 4: 3 stride-1 convs each + layer4's entry split; layer2: entry + 3 convs on small tiles
    assert sum(n.endswith("_splitk") for n in names) == 7, names
    assert sum(n.endswith("_small") for n in names) == 8, names  # + layer1's 4 convs on small tiles
    y8 = m(x[:8])
    assert torch.equal(y8, m(x[:8]))
    for B in (1, 2, 3, 5):
        assert torch.equal(m(x[:B]), y8[:B]), B
    assert torch.equal(m(x), y_batched)  # B = 9 > 8: batched kernels
    y64 = R.run(synth.synthetic_state_dict(0), xs[:8], torch.float64)
    d = np.abs(y8.cpu().numpy() - y64).reshape(8, -1, 2) * PX
    l2 = np.sqrt((d ** 2).sum(-1))
    db = np.abs(y8.cpu().numpy() - y_batched[:8].cpu().numpy()).max() * PX
    print(f"split-K B<=8: px-L2 max {l2.max():.3e} mean {l2.mean():.3e}; vs batched kernels {db:.3e} px")
    assert l2.max() <= FP16_PX_MAX
    m.set_split_k(0)
    assert torch.equal(m(x[:3]), y_batched[:3])


def test_split_k_latency_mode_fp16x3():
    """The parity-grade latency mode (fp16x3 + pa_detector_set_split_k, conv_splitk.hip X3
    forms): short stem bands, layer1 / layer2 entry on small tiles, every other conv of
    layers 2-4 split-K + splitk_reduce_x3.  Within the 1e-3 px parity bar of the golden
    reference outputs and of the f64 oracle, deterministic, batch-invariant among
    latency-mode batches; larger batches keep the batched X3 kernels' bits."""
    xs = synth.synthetic_frames(7, 9, first=3)
    x = torch.from_numpy(xs).cuda()
    m = model(0, precision="fp16x3")
    y_batched = m(x)
    m.set_split_k(8)
    names = [n for n, _ in m.profile(x[:3])[0]]
    # split: layer2's 3 stride-1 convs, layer3 / layer4 entry + 3 convs each (each conv + its reduce: one name)
    assert sum(n.endswith("_splitk") for n in names) == 11, names
    assert sum(n.endswith("_small") for n in names) == 6, names  # stem, layer1's 4 convs, layer2's entry
    y8 = m(x[:8])
    assert torch.equal(y8, m(x[:8]))
    for B in (1, 3, 5):
        assert torch.equal(m(x[:B]), y8[:B]), B
    assert torch.equal(m(x), y_batched)  # B = 9 > 8: batched kernels
    y64 = R.run(synth.synthetic_state_dict(0), xs[:8], torch.float64)
    err64 = np.abs(y8.cpu().numpy() - y64).max() * PX
    errb = np.abs(y8.cpu().numpy() - y_batched[:8].cpu().numpy()).max() * PX
    print(f"fp16x3 split-K B<=8: max px err vs f64 {err64:.3e}; vs batched X3 kernels {errb:.3e} px")
    assert err64 <= FP32_PX_MAX and errb <= FP32_PX_MAX
    m.set_split_k(0)
    assert torch.equal(m(x[:3]), y_batched[:3])


@pytest.mark.parametrize("idx", range(4))
def test_fp16x3_latency_mode_matches_reference_golden(gold, idx):
    """The golden cases (the reference's own CPU outputs) through the fp16x3 latency mode."""
    name, seed, x = cases()[idx]
    m = model(seed, precision="fp16x3")
    m.set_split_k(x.shape[0])
    y = m(torch.from_numpy(x).cuda()).cpu().numpy()
    err_ref = np.abs(y - gold[f"{name}/y_ref_f32"]).max() * PX
    err64 = np.abs(y - gold[f"{name}/y_oracle_f64"]).max() * PX
    print(f"{name}: fp16x3 latency mode max px err vs ref {err_ref:.3e} vs f64 {err64:.3e}")
    assert err_ref <= FP32_PX_MAX and err64 <= FP32_PX_MAX


def test_cpu_input_like_streaming_py():
    """streaming.py:126-128 calls the model on a CPU tensor: result comes back on CPU."""
    x = synth.synthetic_frames(0, 1)
    m = model(0, precision="fp32")
    y = m(torch.from_numpy(x))
    assert y.device.type == "cpu" and y.shape == (1, 16)
    y64 = R.run(synth.synthetic_state_dict(0), x, torch.float64)
    assert np.abs(y.numpy() - y64).max() * PX <= FP32_PX_MAX


def test_empty_batch_and_reload():
    m = model(0)
    y = m(torch.zeros((0, 4, 256, 256), device="cuda"))
    assert y.shape == (0, 16)
    x = torch.from_numpy(synth.synthetic_frames(0, 2)).cuda()
    y0 = m(x)
    m.load_state_dict({k: torch.from_numpy(np.asarray(v)) for k, v in synth.synthetic_state_dict(7).items()})
    y7 = m(x)  # weights re-uploaded after load_state_dict
    assert not torch.equal(y0, y7)


def test_refresh_weights_after_data_write():
    """Writes through .data bypass the version counters the weight fingerprint reads;
    refresh_weights() re-uploads."""
    m = model(0)
    x = torch.from_numpy(synth.synthetic_frames(0, 2)).cuda()
    y0 = m(x)
    m.resnet.fc.bias.data[0] += 1.0
    m.refresh_weights()
    y1 = m(x)
    assert not torch.equal(y0[:, 0], y1[:, 0]) and torch.equal(y0[:, 1:], y1[:, 1:])


def test_batch_over_4096_frames_in_chunks():
    """B > 4096 (32-bit activation offsets): the library runs 1024-frame chunks; each frame
    gets the bits it gets in a small batch."""
    x = torch.from_numpy(synth.synthetic_frames(8, 41)).cuda().repeat(100, 1, 1, 1)  # 4100 frames
    m = model(0)
    y = m(x)
    assert y.shape == (4100, 16)
    for i in (0, 1023, 1024, 4095, 4099):
        assert torch.equal(m(x[i:i + 1])[0], y[i]), i


def test_postprocess_matches_validate_py():
    y = torch.rand(4, 16, device="cuda") * 2 - 1
    t = torch.rand(4, 16, device="cuda") * 2 - 1
    px, loss = denormalize_pixel_coordinates(y, 256, 256, target=t)
    # kornia denormalize_pixel_coordinates, operation for operation (oracle.resnet_ref.denormalize_f32)
    factor = torch.tensor(2.0) / (torch.tensor([256.0, 256.0]) - 1).clamp(1e-8)
    ref_px = torch.tensor(1.0) / factor.cuda() * (y.reshape(4, 8, 2) + 1)
    assert torch.equal(px, ref_px)
    np.testing.assert_array_equal(px.cpu().numpy(), R.denormalize_f32(y.cpu().numpy()))
    ref_loss = torch.nn.SmoothL1Loss(beta=1.0, reduction="none")(t, y)
    assert torch.allclose(loss, ref_loss, atol=0, rtol=0)


def test_profile_reports_every_kernel():
    m = model(0)
    x = torch.from_numpy(synth.synthetic_frames(0, 8)).cuda()
    prof, y = m.profile(x)
    names = [n for n, _ in prof]
    assert names[0] == "stem_conv7x7_pool" and names[-1] == "avgpool_fc"  # fp16: stem + maxpool fused
    assert len(names) == 1 + 4 + 4 + 4 + 4 + 1  # stride-2 conv1 + 1x1 downsample fused
    assert names[5].startswith("conv3x3s2")
    assert torch.equal(y, m(x))
    try:
        m.set_variants({7: 3, 4: 65})  # avgpool + fc fused into layer4's last conv (one-K-group form)
        names_fused = [n for n, _ in m.profile(x)[0]]
    finally:
        m.set_variants({})
    assert names_fused[-1] == "conv3x3x_l4_avgpool_fc" and len(names_fused) == len(names) - 1
    m.precision = "fp32"
    prof32, _ = m.profile(x)
    assert [n for n, _ in prof32][:2] == ["stem_conv7x7", "maxpool"]


def test_fp16x3_stride2_variants_agree_bit_for_bit(gold):
    """fp16x3 stride-2 entries: the row-split kernel (conv_s2w.h X3; layers 2 and 3 until round 5:
    variant 59) against its one- / two-tile workgroup variant (same sum order: bit for bit);
    conv_s2x.h's 8-wave tile (variant 45) against its 4-wave one (44), bit for bit; and the kernel
    families (taps summed in other orders; shipped: layer2 on conv_x3s2v.hip, layer3 on
    conv_x3s2k.hip) within f32 rounding, at the golden outputs' 1e-3 px."""
    m = model(0, precision="fp16x3")
    x = torch.from_numpy(synth.synthetic_frames(4, 5)).cuda()

    def run(v):
        try:
            m.set_variants({6: v})
            return m(x)
        finally:
            m.set_variants({})

    y0, y59, y46, y45, y44 = m(x), run(59), run(46), run(45), run(44)
    assert torch.equal(y59, y46)
    assert torch.equal(y45, y44)
    assert (y0 - y45).abs().max().item() * PX <= 1e-4
    assert (y0 - y59).abs().max().item() * PX <= 1e-4
    name, seed, xg = cases()[0]
    mg = model(seed, precision="fp16x3")
    for v in (0, 45, 59):
        try:
            mg.set_variants({6: v} if v else {})
            y = mg(torch.from_numpy(xg).cuda()).cpu().numpy()
        finally:
            mg.set_variants({})
        assert np.abs(y - gold[f"{name}/y_ref_f32"]).max() * PX <= FP32_PX_MAX


@pytest.mark.parametrize("B", [1, 5, 64, 70])
def test_fp16x3_entries_vgpr_weights(gold, B):
    """fp16x3 layer2 / layer3 entries with the hi / lo weights in VGPRs (shipped from round 6; 6:57
    the same kernels: layer2 on conv_x3s2v.hip, layer3 on conv_x3s2k.hip, its K sum split over
    the waves by input block): the products summed group by group (x_hi w_hi, x_hi w_lo, x_lo w_hi)
    instead of conv_s2w.h X3's plane by plane, so within f32 rounding of round 5's kernels (6:59,
    1e-4 px, as the two stride-2 families above); the timestamping (6:58) and deferred-store (6:60)
    forms bit-identical; deterministic; and at the golden outputs' 1e-3 px (the reference's own CPU
    keypoints and the f64 oracle)."""
    m = model(0, precision="fp16x3")
    x = torch.from_numpy(synth.synthetic_frames(4, B)).cuda()
    y0 = m(x)
    buf = torch.zeros(24 * 65536, dtype=torch.int64, device="cuda")
    try:
        m.set_variants({6: 59})  # round 5's conv_s2w.h X3 entries
        y5 = m(x)
        m.set_variants({6: 57})
        y1, y1b = m(x), m(x)
        m.set_variants({6: 60})  # layer2 with deferred stores
        y3 = m(x)
        m.set_variants({6: 62})  # layer3 with deferred stores
        y4 = m(x)
        m.set_variants({6: 58})
        m.set_trace(buf)
        y2 = m(x)
    finally:
        m.set_trace(None)
        m.set_variants({})
    assert (y5 - y1).abs().max().item() * PX <= 1e-4
    assert torch.equal(y0, y1) and torch.equal(y1, y1b) and torch.equal(y1, y2) and torch.equal(y1, y3)
    assert torch.equal(y1, y4)
    name, seed, xg = cases()[3]
    mg = model(seed, precision="fp16x3")
    try:
        mg.set_variants({6: 57})
        y = mg(torch.from_numpy(xg).cuda()).cpu().numpy()
    finally:
        mg.set_variants({})
    assert np.abs(y - gold[f"{name}/y_ref_f32"]).max() * PX <= FP32_PX_MAX
    assert np.abs(y - gold[f"{name}/y_oracle_f64"]).max() * PX <= FP32_PX_MAX


@pytest.mark.parametrize("B,small", [(64, False), (5, False), (3, True)])
def test_fp16x3_stem_role_split_is_bit_identical(B, small):
    """fp16x3 stem: the role-split kernel (shipped) against the all-waves form (variant 30):
    the same products in the same order per accumulator, so the pooled (hi, lo) map and the
    keypoints are bit for bit equal -- batched (16-row bands) and in the latency mode (2-row
    bands)."""
    m = model(0, precision="fp16x3")
    if small:
        m.set_split_k(8)
    x = torch.from_numpy(synth.synthetic_frames(6, B)).cuda()
    y0 = m(x)
    try:
        m.set_variants({0: 30})
        y1 = m(x)
    finally:
        m.set_variants({})
    assert torch.equal(y0, y1)


@pytest.mark.parametrize("precision", ["fp16", "fp16x3"])
def test_split_k_reduce_forms_bit_identical(precision):
    """The split-K reduces with the split count at compile time (every partial loaded before
    the first add) against the runtime-count loop (variant 7:5): same sum order, same bits."""
    m = model(0, precision=precision)
    m.set_split_k(8)
    x = torch.from_numpy(synth.synthetic_frames(8, 3)).cuda()
    y0 = m(x)
    try:
        m.set_variants({7: 5})
        y1 = m(x)
    finally:
        m.set_variants({})
    assert torch.equal(y0, y1)


@pytest.mark.parametrize("B", [1, 3, 64])
def test_fp16x3_layer1_vgpr_weight_kernel_bit_identical(B):
    """fp16x3 layer1 on conv_x3v.hip (shipped: weights hi / lo in VGPRs, persistent 8-row tiles)
    sums its products in conv_gx X3's merged-step order (variant 1:91) and splits the same way:
    bit-identical; so are its plain convs with their stores at the tile end (1:90; shipped from round
    6: deferred into the next tile's K loop) and its residual convs with every store at the tile end
    (1:97; shipped from round 6: the last row deferred)."""
    m = model(0, precision="fp16x3")
    x = torch.from_numpy(synth.synthetic_frames(5, B)).cuda()
    y0 = m(x)
    try:
        m.set_variants({1: 91})
        y1 = m(x)
        m.set_variants({1: 90})
        y2 = m(x)
        m.set_variants({1: 98})  # the residual convs' stores deferred as well
        y3 = m(x)
        m.set_variants({1: 97})  # the residual convs' stores all at the tile end
        y4 = m(x)
        m.set_variants({1: 99})  # the residual convs' last two rows deferred (VGPRs)
        y5 = m(x)
    finally:
        m.set_variants({})
    assert torch.equal(y0, y1)
    assert torch.equal(y0, y2)
    assert torch.equal(y0, y3)
    assert torch.equal(y0, y4) and torch.equal(y0, y5)


def test_fp16x3_merged_steps_match_three_block_form(gold):
    """fp16x3 3x3 s1 convs: the merged x_hi steps (shipped: x_hi w_hi and x_hi w_lo from one
    fragment read) against three virtual blocks per 64 channels (variant 70).  The f32
    accumulation order differs (products interleaved per tap), so agreement is to f32
    rounding, far below the 1e-3 px bar; both meet the bar against the golden outputs."""
    name, seed, xn = cases()[0]
    m = model(seed, precision="fp16x3")
    x = torch.from_numpy(xn).cuda()
    xb = torch.from_numpy(synth.synthetic_frames(4, 64)).cuda()
    y0, yb0 = m(x), m(xb)
    try:
        m.set_variants({1: 70, 2: 70, 3: 70, 4: 70})
        y1, yb1 = m(x), m(xb)
    finally:
        m.set_variants({})
    assert (y0 - y1).abs().max().item() * PX <= 1e-4
    assert (yb0 - yb1).abs().max().item() * PX <= 1e-4
    for y in (y0, y1):
        assert np.abs(y.cpu().numpy() - gold[f"{name}/y_ref_f32"]).max() * PX <= FP32_PX_MAX


@pytest.mark.parametrize("B", [1, 3, 64])
def test_kernel_variants_agree_bit_for_bit(B):
    """The persistent kernels (layer1 weight-resident conv, stride-2 + downsample; round 6: the
    layer2 entry with its weights in VGPRs, conv_s2v.hip, against conv_s2w.h, variant 6:40)
    and the one-tile-per-workgroup kernels they replace accumulate in the same order:
    identical outputs, at batches below and above one tile per CU.  (Stem variants 10
    and 16 are version 3 of the stem at two band heights.)  The shipped layer2 / layer3
    stride-2 entries (conv_s2w.h, row-split patch) sum the conv's taps in another order
    (kh = 1, 0, 2) than conv_s2x.h and the one-tile kernel (kh = 0, 1, 2): they agree bit for
    bit with their own variants, and the conv_s2x.h forms (variant 6:10 = conv_s2x.h on
    every entry) with each other; the two orders stay within 0.05 px."""
    m = model(0)
    x = torch.from_numpy(synth.synthetic_frames(2, B)).cuda()

    def run(vs):
        try:
            m.set_variants(dict(vs))
            return m(x)
        finally:
            m.set_variants({})

    y0 = m(x)
    y65 = run({4: 65})  # layer4 in one K group of 8 waves (the shipped form, named explicitly)
    assert torch.equal(y0, y65)
    ys2x = run({6: 10})
    assert (y0 - ys2x).abs().max().item() * PX <= 0.05
    sets = (
        (((1, 3), (2, 1), (3, 1), (4, 1), (0, 10)), y65),  # 4:1 = 4:65 with a barrier every 2 steps
        (((1, 30), (7, 1)), y0),  # layer1: register-staged kernel on every conv; the generic head
        (((1, 32),), y0),  # layer1: the one-tile patch kernel (independent of the shipped LDS-DMA kernel)
        (((7, 3), (4, 65)), y65),  # avgpool + fc fused into layer4's last conv instead of head_fp16
        (((0, 16),), y0),  # stem: version 3 (every wave convolves and moves rows) vs the shipped role split
        (((0, 31),), y0),  # stem: bias as the first MFMA's accumulator input (BR) alone
        (((0, 33),), y0),  # stem: IL alone
        (((0, 34),), y0),  # stem: neither BR nor IL (round 4's form; shipped = both)
        (((1, 60),), y0),  # layer1: conv_c64d.hip (weights resident in LDS; shipped until round 5)
        (((1, 80),), y0),  # layer1: conv_c64v.hip 16-row tiles on every conv
        (((1, 81),), y0),  # layer1: conv_c64v.hip 8-row tiles, two 4-wave workgroups per CU, on every conv
        (((1, 83),), y0),  # layer1: conv_c64v.hip 8-row tiles, tiles after the first from per-XCD counters
        (((1, 93),), y0),  # layer1: conv_c64v.hip with deferred stores (plain: staged in LDS, residual: in VGPRs)
        (((1, 96),), y0),  # layer1: deferred stores on the plain convs only
        (((1, 99),), y0),  # layer1: the plain convs' last row deferred
        (((0, 30), (1, 69)), y0),  # stem bands in XCD-grouped order; conv_c64d tiles in the plain order (same arithmetic)
        (((6, 40),), y0),  # conv_s2w on layers 2 and 3 (round 5's entries) vs conv_s2v (layer2, weights in VGPRs)
        (((6, 48),), y0),  # layer2's entry with its stores at the tile end (shipped: deferred); layer4's in the 2 x 4 XCD split
        (((6, 41),), y0),  # conv_s2w: layer2 one tile per workgroup, layer3 prefetch distance 2
        (((6, 42),), y0),  # conv_s2w: layer2 prefetch distance 2
        (((6, 44),), y0),  # conv_s2w: XCD-aware order off
        (((6, 3),), ys2x),  # the one-tile stride-2 kernel (conv_s2.hip) on every entry
        (((6, 11),), ys2x),  # conv_s2x: one tile per workgroup (layer2: the round-2a 8x16 kernel)
        (((6, 26),), ys2x),  # conv_s2x multi-tile workgroups: layer2 4 waves of 32x64; layer3 as shipped
        (((6, 27),), ys2x),  # conv_s2x layer2 prefetch distance 3; layer3 two 4x16 tiles per workgroup
    )
    for vs, ref in sets:
        assert torch.equal(run(vs), ref), vs


@pytest.mark.parametrize("B", [1, 3, 64, 70])
def test_s2k_entries_vgpr_weights_k_split(B):
    """Layers 3 and 4's stride-2 entries on conv_s2k.hip (weights in VGPRs, the K sum split over
    the waves by 64-channel input block and the partials added in block order; variant 6:55):
    another f32 summation order than the LDS-ring kernels, so within 0.05 px of them (the bound
    the two ring orders share, test_kernel_variants_agree_bit_for_bit); its timestamping form
    (6:56) is bit-identical; deterministic over repeats; odd batches (70: a partial round of
    tiles) included."""
    m = model(0)
    x = torch.from_numpy(synth.synthetic_frames(4, B)).cuda()
    y0 = m(x)
    buf = torch.zeros(24 * 65536, dtype=torch.int64, device="cuda")
    try:
        m.set_variants({6: 55})
        y1 = m(x)
        y1b = m(x)
        m.set_variants({6: 56})
        m.set_trace(buf)
        y2 = m(x)
    finally:
        m.set_trace(None)
        m.set_variants({})
    assert (y0 - y1).abs().max().item() * PX <= 0.05
    assert torch.equal(y1, y1b)
    assert torch.equal(y1, y2)
    assert int((buf != 0).sum().item()) > 0  # the stamps were written


@pytest.mark.parametrize("B", [1, 3, 64, 70])
def test_s1k_layer2_vgpr_weights_k_split(B):
    """Layer2's three 3x3 stride-1 convs on conv_s1k.hip (weights in VGPRs, the K sum split over the
    waves by 64-channel input block, partials added in block order; variant 2:80): another f32
    summation order than conv_gx.h, so within 0.05 px of it; its timestamping form (2:81) is
    bit-identical; deterministic over repeats; odd batches (70: a partial round of tiles) included."""
    m = model(0)
    x = torch.from_numpy(synth.synthetic_frames(6, B)).cuda()
    y0 = m(x)
    buf = torch.zeros(24 * 65536, dtype=torch.int64, device="cuda")
    try:
        m.set_variants({2: 80})
        y1 = m(x)
        y1b = m(x)
        m.set_variants({2: 81})
        m.set_trace(buf)
        y2 = m(x)
    finally:
        m.set_trace(None)
        m.set_variants({})
    assert (y0 - y1).abs().max().item() * PX <= 0.05
    assert torch.equal(y1, y1b)
    assert torch.equal(y1, y2)
    assert int((buf != 0).sum().item()) > 0  # the stamps were written


@pytest.mark.parametrize("B", [1, 3, 64, 70])
def test_gx_k_split_variants(B):
    """conv_gx.h's K split over two wave groups (KS = 2: group kg sums half-step kg of every step,
    the groups swap tile halves through LDS and finish (group 0's partial) + (group 1's)): shipped on
    layer4's fp16x3 3x3 s1 convs (against the one-K-group form 4:74); in fp16 (4:67, faster per launch,
    slower over whole forwards) and on layer3 (3:66) measured and not shipped.  Another f32 summation order, so within
    0.05 px in fp16 and 1e-4 px in fp16x3 (whose own error vs the f64 oracle is ~7e-5 px); every form
    deterministic; the shipped fp16x3 within 1e-3 px of the f64 oracle; odd batches (a half-filled
    image pair on layer4) included."""
    x = torch.from_numpy(synth.synthetic_frames(6, B)).cuda()
    m = model(0)
    y0 = m(x)
    assert torch.equal(y0, m(x))
    try:
        for v in ({3: 66}, {4: 67}):
            m.set_variants(v)
            y1 = m(x)
            assert torch.equal(y1, m(x)), v
            assert (y0 - y1).abs().max().item() * PX <= 0.05, v
    finally:
        m.set_variants({})
    m3 = model(0, precision="fp16x3")
    z0 = m3(x)
    assert torch.equal(z0, m3(x))
    try:
        for v in ({4: 74}, {4: 72}):
            m3.set_variants(v)
            z1 = m3(x)
            assert torch.equal(z1, m3(x)), v
            assert (z0 - z1).abs().max().item() * PX <= (0.0 if v[4] == 72 else 1e-4), v
    finally:
        m3.set_variants({})
    y64 = R.run(synth.synthetic_state_dict(0), synth.synthetic_frames(6, B), torch.float64)
    assert np.abs(z0.cpu().numpy() - y64).max() * PX <= FP32_PX_MAX


def test_forward_into_out_buffer():
    """forward(x, out=buf) writes the same keypoints into buf (bench.py's step) and rejects a bad buffer."""
    m = model(0)
    x = torch.from_numpy(synth.synthetic_frames(0, 4)).cuda()
    ref = m(x)
    buf = torch.full((2, 4, 16), float("nan"), device="cuda")
    got = m(x, out=buf[1])
    assert got.data_ptr() == buf[1].data_ptr()
    assert torch.equal(buf[1], ref) and torch.isnan(buf[0]).all()
    with pytest.raises(RuntimeError):
        m(x, out=torch.empty((4, 16), dtype=torch.float16, device="cuda"))
    with pytest.raises(RuntimeError):
        m(x, out=torch.empty((16, 4), device="cuda").t())


def test_fused_head_repeats_and_batch_changes():
    """The fused head (variant 7:3) keeps per-image-pair counters that return to zero after
    every launch: repeated forwards, odd batches and a batch larger than the last reserve all
    give the separate head's bits."""
    m = model(1)
    for B in (2, 5, 64, 7, 130):
        x = torch.from_numpy(synth.synthetic_frames(3, B)).cuda()
        try:
            m.set_variants({4: 65})  # layer4 in one K group: the form the fused head extends
            ref = m(x)
            m.set_variants({7: 3, 4: 65})
            ys = [m(x) for _ in range(3)]
        finally:
            m.set_variants({})
        for y in ys:
            assert torch.equal(y, ref), B


@pytest.mark.parametrize("precision", ["fp32", "fp16"])
def test_reserve_is_clamped_to_one_chunk(precision):
    """pa_detector_reserve clamps to the 1,024-frame chunk the forward runs in: reserving a
    configs[2]-sized batch (24,000 frames; unclamped ~176 GB of f32 workspace) succeeds, and
    a 4,100-frame forward (five chunks) then matches the same frames forwarded alone."""
    m = KeypointCNN(num_channels=4, precision=precision)
    m.load_state_dict({k: torch.from_numpy(np.asarray(v)) for k, v in synth.synthetic_state_dict(0).items()})
    m.reserve(24000)
    x = torch.from_numpy(synth.synthetic_frames(0, 8)).cuda()
    xs = x.repeat(513, 1, 1, 1)[:4100].contiguous()
    y = m(xs)
    ref = m(x)
    for off in (0, 1024, 2048, 4096):
        assert torch.equal(y[off:off + 4], ref[(off % 8):(off % 8) + 4]), off
