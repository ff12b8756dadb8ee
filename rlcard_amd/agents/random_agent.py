"""RandomAgent with rlcard's semantics (rlcard/agents/random_agent.py:4-47): a uniform pick over the legal ids from
numpy's GLOBAL RandomState, so `np.random.seed(s)` reproduces the reference's choices (config 1 of BASELINE.json)."""
import numpy as np


class RandomAgent(object):
    def __init__(self, num_actions):
        self.use_raw = False
        self.num_actions = num_actions

    @staticmethod
    def step(state):
        return np.random.choice(list(state['legal_actions'].keys()))

    def eval_step(self, state):
        legal = list(state['legal_actions'].keys())
        p = 1.0 / len(legal)
        info = {'probs': {state['raw_legal_actions'][i]: p for i in range(len(legal))}}
        return self.step(state), info
