from .fd_return import FDReturn, FDBatch  # noqa: F401
from .fd_state import FDState  # noqa: F401
from .finite_differences import FiniteDifferences  # noqa: F401
