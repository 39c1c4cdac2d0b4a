"""GPU parity of the validation loss statistics (validate.py:162-168) against torch/numpy.

Tolerances: min, max and median bit-exact (selection, no arithmetic); mean and stdev are
f64 sums on the device, compared with numpy f64 at rtol 1e-9 (summation order differs)."""
import numpy as np
import pytest
import torch

from perseus_amd.detector import denormalize_pixel_coordinates, loss_statistics

pytestmark = pytest.mark.gpu


def check(x: torch.Tensor):
    st = loss_statistics(x.cuda())
    v = x.reshape(-1).double().numpy()
    assert st["min"] == float(x.min()) and st["max"] == float(x.max())
    assert st["median"] == float(torch.median(x.reshape(-1)))  # lower middle element
    np.testing.assert_allclose(st["mean"], v.mean(), rtol=1e-9, atol=0)
    if v.size > 1:
        np.testing.assert_allclose(st["std"], v.std(ddof=1), rtol=1e-9, atol=1e-300)
    else:
        assert np.isnan(st["std"]) and torch.isnan(x.reshape(-1).std())
    return st


@pytest.mark.parametrize("n", [1, 2, 3, 16, 1024, 16 * 64 + 3, 1_000_003])
def test_random_lengths(n):
    g = torch.Generator().manual_seed(n)
    check(torch.rand(n, generator=g) * 3.0)


def test_ties_negatives_and_unaligned_view():
    g = torch.Generator().manual_seed(1)
    x = torch.randint(-5, 6, (40_001,), generator=g).float() + 0.5  # many ties, both signs, no zeros
    check(x)
    base = torch.rand(10_001, generator=g).cuda()
    st = loss_statistics(base[1:])  # 4-byte offset: the scalar tail path
    ref = base[1:].cpu()
    assert st["median"] == float(torch.median(ref)) and st["max"] == float(ref.max())


def test_validate_py_pipeline():
    """SmoothL1 losses from the device post-process, then the statistics, as validate.py:130-168."""
    g = torch.Generator().manual_seed(2)
    y = (torch.rand(64, 16, generator=g) * 2 - 1).cuda()
    t = (torch.rand(64, 16, generator=g) * 2 - 1).cuda()
    _, loss = denormalize_pixel_coordinates(y, 256, 256, target=t)
    ref = torch.nn.SmoothL1Loss(beta=1.0, reduction="none")(t.cpu(), y.cpu()).reshape(-1)
    st = check(loss.cpu())
    assert st["median"] == float(torch.median(ref))
    np.testing.assert_allclose(st["mean"], float(ref.double().mean()), rtol=1e-6)


@pytest.mark.parametrize("n", [16, 1024, 64 * 16 * 40])
def test_printed_f32_values_match_torch_f32(n):
    """validate.py:165 prints torch f32 reductions: the f32 mean / stdev agree with torch's
    own f32 results to 2 ulps (torch's summation order differs from the device's f64 sums
    rounded once), and min / max / median bit for bit; the report has validate.py's form."""
    from perseus_amd.detector import validation_report

    g = torch.Generator().manual_seed(n)
    x = torch.nn.SmoothL1Loss(beta=1.0, reduction="none")(torch.rand(n, generator=g) * 2 - 1,
                                                          torch.rand(n, generator=g) * 2 - 1)
    st = loss_statistics(x.cuda())
    for key, ref in (("mean_f32", x.mean()), ("std_f32", x.std())):
        ulp = np.spacing(np.float32(ref.item()))
        assert abs(st[key] - ref.item()) <= 2 * ulp, (key, st[key], ref.item())
    rep = validation_report(x.cuda()).splitlines()
    assert rep[1] == "Validation Loss" and rep[3] == f"Min: {x.min()}" and rep[5] == f"Median: {torch.median(x)}"


def test_empty_raises():
    with pytest.raises(RuntimeError):
        loss_statistics(torch.empty(0, device="cuda"))
