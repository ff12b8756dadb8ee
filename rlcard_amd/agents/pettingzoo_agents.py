"""Agents for envs with PettingZoo's AEC protocol (rlcard/agents/pettingzoo_agents.py:38-43): the agent sees the AEC
observation dict through wrap_state. Only RandomAgentPettingZoo: the reference's DQN / NFSP PettingZoo agents wrap
learners that are outside this engine's scope."""
from ..utils import wrap_state
from .random_agent import RandomAgent


class RandomAgentPettingZoo(RandomAgent):
    def step(self, state):
        return super().step(wrap_state(state))

    def eval_step(self, state):
        return super().eval_step(wrap_state(state))
