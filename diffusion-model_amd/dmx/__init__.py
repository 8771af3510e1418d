"""dmx — MI355X-native CFG latent-diffusion sampler (runtime package).

``dmx`` holds the native runtime (libdmx.so + its ctypes binding); the
reference-compatible drop-in modules (``diff``, ``entityCsvSampler``,
``models.*``, ``utils``) live beside it in ``diffusion-model_amd/``.
"""
from ._lib import DmxError, DmxUnavailable, load  # noqa: F401

__all__ = ["DmxError", "DmxUnavailable", "load"]
