"""fdr -- MI355X-native finite-difference rollout + gradient engine (runtime layer).

Importing ``fdr`` loads libfdr.so (the HIP kernels, gfx950) and fails loudly if it is missing.
"""
from ._lib import FDRError, LIB_PATH, version  # noqa: F401
from . import engine  # noqa: F401
