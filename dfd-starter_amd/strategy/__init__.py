from .strategy_handler import StrategyHandler  # noqa: F401
