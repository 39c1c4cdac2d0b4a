"""Host-side logic of the drop-in surfaces (no GPU)."""
import numpy as np
import pytest
import torch

from perseus_amd import smoother, synth
from perseus_amd.detector import KeypointCNN


def test_keypointcnn_surface_matches_reference_keys():
    m = KeypointCNN(num_channels=4)
    assert (m.n_keypoints, m.num_channels, m.H, m.W) == (8, 4, 256, 256)
    keys = list(m.state_dict().keys())
    assert keys == list(synth.resnet18_shapes(4, 8).keys())
    assert len(keys) == 122


def test_load_state_dict_after_module_strip_like_validate():
    m = KeypointCNN(num_channels=4)
    st = synth.synthetic_state_dict(0)
    sd = {"module." + k: torch.from_numpy(np.asarray(v)) for k, v in st.items()}
    for key in list(sd.keys()):  # validate.py:93-97
        if "module." in key:
            sd[key.replace("module.", "")] = sd.pop(key)
    m.load_state_dict(sd)
    np.testing.assert_array_equal(m._blob(), synth.weight_blob(st))


def test_rgb_model_and_bad_shapes():
    m = KeypointCNN(num_channels=3)
    assert m.state_dict()["resnet.conv1.weight"].shape == (64, 3, 7, 7)
    with pytest.raises(ValueError):
        KeypointCNN(H=128, W=128)
    with pytest.raises(RuntimeError):
        m(torch.zeros(1, 4, 256, 256))  # wrong channel count: reference raises from conv2d too


def test_inference_only():
    m = KeypointCNN()
    with pytest.raises(NotImplementedError):
        m.train()
    assert m.eval() is m


def test_containers_and_factor_surface():
    v = smoother.Values()
    v.insert(0, smoother.Pose3(np.eye(3), [1, 2, 3]))
    v.insert(1, np.array([1.0, 2.0, 3.0]))
    with pytest.raises(KeyError):
        v.insert(1, np.zeros(3))
    assert np.allclose(v.atPose3(0).matrix()[:3, 3], [1, 2, 3])
    nm = smoother.noiseModel.Diagonal.Sigmas(np.array([0.1] * 6))
    f = smoother.PoseDynamicsFactor(0, 1, 2, 3, nm, 0.1)
    assert f.keys() == [0, 1, 2, 3] and f.vel_frame == "world"
    with pytest.raises(AssertionError):
        smoother.PoseDynamicsFactor(0, 1, 2, 3, nm, 0.1, vel_frame="camera")
    K = smoother.Cal3_S2(280, 280, 0, 128, 128)
    p = smoother.KeypointProjectionFactor(0, nm, K, [1, 2], [0, 0, 0])
    assert p.pixel is None and p.keys() == [0]



def test_csrc_digest_ignores_comments_not_code(tmp_path, monkeypatch):
    """bench.csrc_digest keys the committed PMC records (profiles/pmc_*.json): a comment-only
    edit of a kernel source keeps the record valid, a code edit invalidates it."""
    import bench

    src = tmp_path / "perseus_amd" / "csrc"
    src.mkdir(parents=True)
    f = src / "k.hip"
    monkeypatch.setattr(bench, "ROOT", str(tmp_path))
    f.write_text("int a = 1;  // one\n/* block\n comment */ int b = 2;\n")
    d0 = bench.csrc_digest()
    f.write_text("// a new header line\nint a = 1;  // ONE\nint b = 2;   /* moved */\n")
    assert bench.csrc_digest() == d0
    f.write_text("int a = 1;\nint b = 3;\n")
    assert bench.csrc_digest() != d0
    # line breaks end preprocessor directives: joining two lines is a code change
    f.write_text("#define N 4\nint c = N;\n")
    d1 = bench.csrc_digest()
    f.write_text("#define N 4 int c = N;\n")
    assert bench.csrc_digest() != d1
    # a "//" inside a string literal is code, not a comment
    f.write_text('const char* s = "a//b";\n')
    d2 = bench.csrc_digest()
    f.write_text('const char* s = "a//c";\n')
    assert bench.csrc_digest() != d2


def test_timing_only_variants_rejected_by_release_library():
    """The wrong-result timing variants (csrc/common.h PA_TIMING_VARIANTS) are not in the release
    library: pa_detector_debug_set_variant refuses their ids before it looks at the handle, so no
    public call can select them.  Shipped-alternative ids pass that check and
    then fail only on the NULL handle.  No GPU call is made."""
    from perseus_amd import _lib

    L = _lib.lib()
    assert L.pa_debug_timing_variants_built() == 0
    for layer, v in ((0, 26), (1, 87), (1, 89), (1, 66), (1, 38), (3, 60), (4, 64)):
        assert L.pa_detector_debug_set_variant(None, layer, v) < 0
        assert b"timing-only" in L.pa_last_error(), (layer, v)
    for layer, v in ((0, 34), (1, 80), (1, 60), (3, 53), (4, 58), (6, 41)):
        assert L.pa_detector_debug_set_variant(None, layer, v) < 0
        assert b"null detector" in L.pa_last_error(), (layer, v)
