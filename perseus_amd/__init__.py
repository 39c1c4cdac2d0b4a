"""perseus_amd — MI355X (gfx950) implementation of perseus's keypoint-inference path.

Drop-in surfaces (see DESIGN.md / INTEGRATION.md):
  * perseus_amd.detector.KeypointCNN         <- perseus/detector/models.py:6-40
  * perseus_amd.smoother.{PoseDynamicsFactor, ConstantVelocityFactor,
    KeypointProjectionFactor} + batched linearize_*  <- perseus/smoother/factors.py
The compute lives in libperseus_amd.so (HIP, C ABI: include/perseus_amd.h).
"""

__version__ = "0.1.0"


def __getattr__(name):  # lazy: importing the package does not load torch or the .so
    if name == "KeypointCNN":
        from .detector import KeypointCNN

        return KeypointCNN
    raise AttributeError(name)
