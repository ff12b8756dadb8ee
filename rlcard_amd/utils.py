"""Host utilities mirroring rlcard/utils/utils.py that examples call around the env path."""
import random

import numpy as np


def set_seed(seed):
    """utils.py set_seed: seeds numpy's and Python's global generators (and torch's when importable)."""
    if seed is not None:
        np.random.seed(seed)
        random.seed(seed)
        try:
            import torch
            torch.manual_seed(seed)
        except ImportError:
            pass
