from .random_agent import RandomAgent  # noqa: F401
from .cfr_agent import CFRAgent  # noqa: F401
from .dmc_agent import DMCAgent, DMCModel, DMCNet, ActorBuffers, DMCActor  # noqa: F401
