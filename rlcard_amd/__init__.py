"""rlcard_amd -- MI355X-native batched card-game environments (Blackjack, Leduc Hold'em, Limit Hold'em,
No-limit Hold'em, DouDizhu).

Drop-in for the reference's env path: rlcard_amd.make(env_id, config) returns an Env with rlcard's
reset/step/run/get_state/get_payoffs API (rlcard/envs/env.py), and rlcard_amd.VecEnv runs N such envs in lockstep
on one GPU through the C ABI in include/cardsim.h (HIP kernels for gfx950, rlcard_amd/csrc/).
"""
__version__ = '0.1.0'

from .vec import VecEnv, legal_mask, legal_ids  # noqa: F401
from .envs import make, register  # noqa: F401
