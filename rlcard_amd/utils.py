"""Host utilities mirroring rlcard/utils/utils.py that examples call around the env path (run_random.py, run_cfr.py,
run_rl.py): set_seed, reorganize, remove_illegal, tournament. The batched, on-device forms of reorganize and of the
legal-id lists are VecEnv.transitions / VecEnv.legal_lists (include/cardsim.h)."""
import random

import numpy as np


def set_seed(seed):
    """utils.py:5-18: seeds numpy's and Python's global generators (and torch's when importable)."""
    if seed is not None:
        np.random.seed(seed)
        random.seed(seed)
        try:
            import torch
            torch.manual_seed(seed)
        except ImportError:
            pass


def reorganize(trajectories, payoffs):
    """utils.py:153-179: per player, [state, action, state, ...] -> [state, action, reward, next_state, done]
    transitions; the reward (the player's payoff) and done=True only on the player's last transition."""
    num_players = len(trajectories)
    new_trajectories = [[] for _ in range(num_players)]
    for player in range(num_players):
        seq = trajectories[player]
        for i in range(0, len(seq) - 2, 2):
            if i == len(seq) - 3:
                reward, done = payoffs[player], True
            else:
                reward, done = 0, False
            transition = seq[i:i + 3].copy()
            transition.insert(2, reward)
            transition.append(done)
            new_trajectories[player].append(transition)
    return new_trajectories


def remove_illegal(action_probs, legal_actions):
    """utils.py:181-198: zero the illegal entries; uniform over the legal ids if nothing is left, else renormalise."""
    probs = np.zeros(action_probs.shape[0])
    probs[legal_actions] = action_probs[legal_actions]
    if np.sum(probs) == 0:
        probs[legal_actions] = 1 / len(legal_actions)
    else:
        probs /= sum(probs)
    return probs


def tournament(env, num):
    """utils.py:200-225: average payoff per player over `num` games of env.run (the env's agents set beforehand)."""
    payoffs = [0 for _ in range(env.num_players)]
    counter = 0
    while counter < num:
        _, _payoffs = env.run(is_training=False)
        if isinstance(_payoffs, list):
            for _p in _payoffs:
                for i, _ in enumerate(payoffs):
                    payoffs[i] += _p[i]
                counter += 1
        else:
            for i, _ in enumerate(payoffs):
                payoffs[i] += _payoffs[i]
            counter += 1
    for i, _ in enumerate(payoffs):
        payoffs[i] /= counter
    return payoffs
