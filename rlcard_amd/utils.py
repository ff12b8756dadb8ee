"""Host utilities with the behaviour of rlcard/utils/utils.py that examples call around the env path (run_random.py,
run_cfr.py, run_rl.py): set_seed, reorganize, remove_illegal, tournament. The batched, on-device forms of reorganize
and of the legal-id lists are VecEnv.transitions / VecEnv.legal_lists (include/cardsim.h)."""
import random

import numpy as np


def set_seed(seed):
    """Same effect as utils.py:5-18: numpy's and Python's global generators (and torch's when importable)."""
    if seed is None:
        return
    np.random.seed(seed)
    random.seed(seed)
    try:
        import torch
    except ImportError:
        return
    torch.manual_seed(seed)


def reorganize(trajectories, payoffs):
    """Behaviour of utils.py:153-179. Each player's trajectory alternates states and actions and ends with the final
    state: [s0, a0, s1, a1, ..., sK]. It becomes K transitions [s_k, a_k, reward, s_{k+1}, done], where only the last
    one carries the player's payoff and done=True."""
    out = []
    for p, seq in enumerate(trajectories):
        states, actions = seq[0::2], seq[1::2]
        k_last = len(actions) - 1
        out.append([[states[k], actions[k], payoffs[p] if k == k_last else 0, states[k + 1], k == k_last]
                    for k in range(len(actions)) if k + 1 < len(states)])
    return out


def remove_illegal(action_probs, legal_actions):
    """Behaviour of utils.py:181-198: probabilities restricted to the legal ids and renormalised; uniform over the
    legal ids when they carry no mass."""
    legal = np.asarray(list(legal_actions), dtype=np.int64)
    masked = np.zeros(len(action_probs))
    masked[legal] = np.asarray(action_probs)[legal]
    mass = masked.sum()
    if mass == 0:
        masked[legal] = 1.0 / len(legal)
        return masked
    return masked / mass


def tournament(env, num):
    """Behaviour of utils.py:200-225: mean payoff per player over `num` games of env.run with the env's agents (an
    env whose run returns a list of per-game payoffs counts each of them)."""
    total = np.zeros(env.num_players)
    games = 0
    while games < num:
        _, result = env.run(is_training=False)
        batch = result if isinstance(result, list) else [result]
        for pay in batch:
            total += np.asarray(pay, dtype=np.float64)[:env.num_players]
            games += 1
    return list(total / games)
