"""PettingZoo's AEC protocol over the engine's envs, so rlcard's PettingZoo helpers (rlcard/utils/pettingzoo_utils.py,
rlcard/agents/pettingzoo_agents.py; here rlcard_amd.utils and rlcard_amd.agents.pettingzoo_agents) run on them without
the pettingzoo package (not installed in this image).

The protocol is the one those helpers use (pettingzoo_utils.py:20-37, examples/pettingzoo/run_rl.py): reset(seed),
agent_iter(), last() -> (observation, reward, termination, truncation, info), step(action), agents / possible_agents
named 'player_<id>', action_space(name).n, observation_space(name)['observation'].shape. An observation is
{'observation': the env's obs (float64 -> float32, int64 -> int8), 'action_mask': int8[num_actions] of the legal ids of
the player to act}. Rewards are 0 until the game ends; then every agent's last() carries its payoff and done = True,
and each agent is stepped once more with None (the dead step), which removes it; the iteration ends when none is left.
This follows PettingZoo's classic RLCard wrapper as documented; it is not checked against pettingzoo itself (parity
unpinned: the package is absent), only against rlcard_amd's own Env (tests/test_pettingzoo.py).
"""
from types import SimpleNamespace

import numpy as np


class AECEnv(object):
    def __init__(self, env_id, config=None):
        from . import make
        self.env = make(env_id, config)
        self.metadata = {'name': env_id}
        self.possible_agents = ['player_%d' % i for i in range(self.env.num_players)]
        self.agents = []
        self.agent_selection = None
        self._legal = []
        self._dtype = None

    @property
    def num_agents(self):
        return len(self.agents)

    def action_space(self, agent):
        return SimpleNamespace(n=self.env.num_actions)

    def observation_space(self, agent):
        shape = tuple(self.env.state_shape[self.possible_agents.index(agent)])
        return {'observation': SimpleNamespace(shape=shape), 'action_mask': SimpleNamespace(shape=(self.env.num_actions,))}

    def _per_agent(self, value):
        return {a: (value() if callable(value) else value) for a in self.possible_agents}

    def reset(self, seed=None, options=None):
        if seed is not None:
            self.env.seed(seed)
        state, pid = self.env.reset()
        dt = np.asarray(state['obs']).dtype
        self._dtype = np.float32 if dt == np.float64 else (np.int8 if dt == np.int64 else dt)
        self.agents = list(self.possible_agents)
        self.agent_selection = self.possible_agents[pid]
        self.rewards = self._per_agent(0)
        self._cumulative_rewards = self._per_agent(0)
        self.terminations = self._per_agent(False)
        self.truncations = self._per_agent(False)
        self.infos = self._per_agent(lambda: {'legal_moves': []})
        self._legal = sorted(state['legal_actions'])

    def observe(self, agent):
        st = self.env.get_state(self.possible_agents.index(agent))
        mask = np.zeros(self.env.num_actions, dtype=np.int8)
        mask[list(self._legal)] = 1
        return {'observation': np.asarray(st['obs']).astype(self._dtype), 'action_mask': mask}

    def last(self, observe=True):
        a = self.agent_selection
        obs = self.observe(a) if observe else None
        return obs, self._cumulative_rewards[a], self.terminations[a], self.truncations[a], self.infos[a]

    def agent_iter(self, max_iter=2 ** 63):
        for _ in range(max_iter):
            if not self.agents:
                return
            yield self.agent_selection

    def step(self, action):
        a = self.agent_selection
        if self.terminations[a] or self.truncations[a]:
            if action is not None:
                raise ValueError('when an agent is done, the only valid action is None')
            self.agents.remove(a)
            del self._cumulative_rewards[a]
            dead = [x for x in self.agents if self.terminations[x] or self.truncations[x]]
            if dead:
                self.agent_selection = dead[0]
            self.rewards = {x: 0 for x in self.agents}
            return
        state, pid = self.env.step(action)
        if self.env.is_over():
            pay = self.env.get_payoffs()
            self.rewards = {x: pay[i] for i, x in enumerate(self.possible_agents)}
            self._legal = []
            self.terminations = self._per_agent(True)
        else:
            self.rewards = self._per_agent(0)
            self._legal = sorted(state['legal_actions'])
        self._cumulative_rewards[a] = 0
        self.agent_selection = self.possible_agents[pid]
        for x in self.agents:
            self._cumulative_rewards[x] += self.rewards[x]

    def close(self):
        pass


def env(env_id, config=None):
    """The AEC env of an engine game id ('leduc-holdem', 'limit-holdem', 'no-limit-holdem', 'doudizhu',
    'blackjack')."""
    return AECEnv(env_id, config)
