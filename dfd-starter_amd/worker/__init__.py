from .agent import Agent  # noqa: F401
from .worker import Worker  # noqa: F401
