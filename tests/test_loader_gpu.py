"""SURVEY.md 8f.3 end to end on the device: dataset items decoded by the native loader
(perseus_amd/data.py over csrc/loader.cpp, one call per batch into pinned host memory), moved
to the GPU and assembled as validate.py:119-121 does (RGB (3,H,W) + depth -> (4,H,W)), then the
detector forward -- against the reference's __getitem__ restated with PIL (oracle/loader_ref.py)
and the f64 oracle forward of those items.  Items bit-exact after the copy; keypoints within
the parity-mode bar (1e-3 px)."""
import numpy as np
import pytest
import torch

from oracle import loader_ref
from oracle import resnet_ref as R
from perseus_amd import synth
from perseus_amd.data import PrunedKeypointDataset
from perseus_amd.detector import KeypointCNN

from test_loader import _write_dataset  # tests/ is on sys.path (rootdir conftest)

pytestmark = pytest.mark.gpu
PX = 127.5


@pytest.mark.parametrize("precision", ["fp16x3", "fp32"])
def test_loaded_batch_through_the_detector(tmp_path, precision):
    n, h, w = 4, 256, 256
    names = _write_dataset(str(tmp_path), n, h, w)
    rng = np.random.default_rng(5)
    asset_ids = rng.integers(0, 3, n)
    px = rng.uniform(0, 256, (n, 8, 2)).astype(np.float32)
    ds = PrunedKeypointDataset.from_index(image_filenames=np.array(names[0]), depth_filenames=np.array(names[1]),
                                          segmentation_filenames=np.array(names[2]), asset_ids=asset_ids,
                                          pixel_coordinates=px, H=h, W=w, root=str(tmp_path))
    batch = ds.load_batch(list(range(n)), n_threads=4, pin_memory=True)
    image = batch["image"].cuda(non_blocking=True)
    depth = batch["depth_image"].cuda(non_blocking=True)
    x = torch.cat((image, depth[..., None, :, :]), dim=-3)  # validate.py:119-121
    refs = [loader_ref.get_item(str(tmp_path), names[0][i].decode(), names[1][i].decode(), names[2][i].decode(),
                                int(asset_ids[i]), torch.from_numpy(px[i])) for i in range(n)]
    x_ref = torch.stack([torch.cat((r["image"], r["depth_image"][None]), dim=0) for r in refs])
    assert torch.equal(x.cpu(), x_ref)
    m = KeypointCNN(num_channels=4, precision=precision)
    m.load_state_dict({k: torch.from_numpy(np.asarray(v)) for k, v in synth.synthetic_state_dict(0).items()})
    y = m.eval()(x).cpu().numpy()
    y64 = R.run(synth.synthetic_state_dict(0), x_ref.numpy(), torch.float64)
    err = np.abs(y - y64).max() * PX
    print(f"{precision}: loaded batch of {n}: max px err vs f64 oracle {err:.3e}")
    assert err <= 1e-3
