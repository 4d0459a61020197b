from .adaptive_omega import AdaptiveOmega  # noqa: F401
from .noise_sources import SharedNoiseTable, SimpleNoiseSource, RNGNoiseSource  # noqa: F401
