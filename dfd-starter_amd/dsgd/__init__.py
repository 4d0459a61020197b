from .dynamic_sgd import DSGD  # noqa: F401
