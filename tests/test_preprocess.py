"""Host-side facts the preprocess kernels rely on (no GPU)."""
import numpy as np


def test_byte_scale_f32_division_equals_numpy_f64_then_float():
    """streaming.py:68-73 scales colour bytes as numpy f64 `/ 255.0` and then `.float()`.
    The stem's fused preprocess (stem.hip load_rows) divides in f32 instead: the correctly
    rounded f32 quotient equals the f64 quotient rounded to f32 for every byte value, so the
    two are the same input bits (no double-rounding case among the 256 values)."""
    b = np.arange(256)
    ref = (b / 255.0).astype(np.float32)
    f32 = b.astype(np.float32) / np.float32(255.0)
    np.testing.assert_array_equal(f32.view(np.uint32), ref.view(np.uint32))
