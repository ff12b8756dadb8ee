"""A small deterministic env with PettingZoo's AEC protocol, test infrastructure for the PettingZoo helpers
(rlcard_amd.utils.*_pettingzoo, tests/golden/gen_golden.py 'pettingzoo'): players act in turn for a number of moves drawn
from the episode seed, observations are small integer vectors, the legal set is a random non-empty subset, and at the
end each player is paid sum-of-its-actions minus the mean. Dead agents are stepped with None and removed, as in
PettingZoo. Not product code: nothing under rlcard_amd imports it."""
import numpy as np


class FakeAEC(object):
    def __init__(self, num_players=3, num_actions=5, obs_len=4, seed=0):
        self.possible_agents = ['player_%d' % i for i in range(num_players)]
        self.num_actions, self.obs_len = num_actions, obs_len
        self._episode = 0
        self._seed = seed

    def reset(self, seed=None, options=None):
        if seed is not None:
            self._seed = seed
        self._rng = np.random.RandomState(self._seed * 1000 + self._episode)
        self._episode += 1
        self.agents = list(self.possible_agents)
        self._moves = int(self._rng.randint(1, 8))
        self._cur = int(self._rng.randint(len(self.agents)))
        self._acts = {a: 0 for a in self.agents}
        self._cum = {a: 0.0 for a in self.agents}
        self._term = {a: False for a in self.agents}
        self.agent_selection = self.agents[self._cur]
        self._new_obs()

    def _new_obs(self):
        self._obs = self._rng.randint(0, 3, size=self.obs_len).astype(np.float32)
        mask = (self._rng.rand(self.num_actions) < 0.6).astype(np.int8)
        mask[self._rng.randint(self.num_actions)] = 1
        self._mask = mask

    def last(self):
        a = self.agent_selection
        return ({'observation': self._obs.copy(), 'action_mask': self._mask.copy()}, self._cum[a], self._term[a], False,
                {})

    def agent_iter(self):
        while self.agents:
            yield self.agent_selection

    def step(self, action):
        a = self.agent_selection
        if self._term[a]:
            assert action is None
            self.agents.remove(a)
            if self.agents:
                self.agent_selection = self.agents[0]
            return
        assert self._mask[action] == 1
        self._acts[a] += int(action)
        self._cum[a] = 0.0
        self._moves -= 1
        self._cur = (self._cur + 1) % len(self.possible_agents)
        self.agent_selection = self.possible_agents[self._cur]
        if self._moves == 0:
            mean = float(np.mean(list(self._acts.values())))
            for x in self.agents:
                self._cum[x] += self._acts[x] - mean
                self._term[x] = True
        self._new_obs()
