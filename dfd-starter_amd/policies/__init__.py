from .policy import Policy  # noqa: F401
from .discrete import DiscretePolicy  # noqa: F401
from .mujoco import MujocoPolicy  # noqa: F401
from .impala import ImpalaPolicy  # noqa: F401
from .atari import AtariPolicy  # noqa: F401
