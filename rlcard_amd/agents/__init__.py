from .random_agent import RandomAgent  # noqa: F401
