"""CFRAgent (rlcard/agents/cfr_agent.py:9-221): chance-sampling CFR on Leduc Hold'em, trained on the GPU.

The reference walks the betting tree with env.step / env.step_back in Python and keeps dicts keyed by the float64
obs bytes. Here train() calls cs_cfr_train (include/cardsim.h): the tree walk, regret / average-policy accumulation
and regret matching run as HIP kernels over dense fp64 tables indexed by the Leduc observation; the dicts
(policy / average_policy / regrets, same keys and values as the reference's) are views built from the tables.

With an rlcard_amd.make('leduc-holdem', {'allow_step_back': True, 'seed': s}) env the deals come from that env's
stream exactly as the reference's env.reset() calls do, so the tables are bit-exact against the reference agent.
With a VecEnv of B envs, every iteration deals B games per player (batched chance sampling).
"""
import ctypes as C
import os

import numpy as np
import torch

from .. import _abi
from ..envs.env import Env
from ..utils import remove_illegal
from ..vec import VecEnv

NUM_INFOSETS = 2700   # ((hand * 4 + public + 1) * 15 + my chips) * 15 + others' chips
NUM_ACTIONS = 4


def infoset_obs(idx):
    """Leduc obs (float64 [36], envs/leducholdem.py:41-71) of a table row."""
    rest, op = divmod(int(idx), 15)
    rest, my = divmod(rest, 15)
    hand, pub = divmod(rest, 4)
    obs = np.zeros(36)
    obs[hand] = 1
    if pub:
        obs[3 + pub - 1] = 1
    obs[6 + my] = 1
    obs[21 + op] = 1
    return obs


def obs_infoset(obs):
    """Table row of a Leduc obs, or -1 for anything that is not one."""
    o = np.asarray(obs)
    if o.shape != (36,) or not np.isin(o, (0, 1)).all():
        return -1
    h, p, m, q = (np.nonzero(o[a:b])[0] for a, b in ((0, 3), (3, 6), (6, 21), (21, 36)))
    if len(h) != 1 or len(p) > 1 or len(m) != 1 or len(q) != 1:
        return -1
    return ((int(h[0]) * 4 + (int(p[0]) + 1 if len(p) else 0)) * 15 + int(m[0])) * 15 + int(q[0])


class CFRAgent(object):
    def __init__(self, env, model_path='./cfr_model'):
        self.use_raw = False
        self.env = env
        self.model_path = model_path
        vec = env._vec if isinstance(env, Env) else env
        if not isinstance(vec, VecEnv) or vec.env_id != 'leduc-holdem':
            raise ValueError('CFRAgent runs on leduc-holdem envs (rlcard_amd.make or VecEnv)')
        self._vecenv = vec
        d = vec.device
        self._policy = torch.full((NUM_INFOSETS, NUM_ACTIONS), 1.0 / NUM_ACTIONS, dtype=torch.float64, device=d)
        self._avg = torch.zeros((NUM_INFOSETS, NUM_ACTIONS), dtype=torch.float64, device=d)
        self._regrets = torch.zeros((NUM_INFOSETS, NUM_ACTIONS), dtype=torch.float64, device=d)
        self._flags = torch.zeros(NUM_INFOSETS, dtype=torch.int32, device=d)
        self._extra_policy = {}     # keys action_probs inserted that are not Leduc observations
        self._host = None
        self.iteration = 0

    # -- training ---------------------------------------------------------------------------------------------
    def train(self, iterations=1):
        """`iterations` x the reference's train() (cfr_agent.py:30-43), on the device."""
        v = self._vecenv
        with torch.cuda.device(v.device):
            _abi.check(_abi.lib().cs_cfr_train(v._h, int(iterations), int(self.iteration), self._ptr(self._policy),
                                               self._ptr(self._avg), self._ptr(self._regrets),
                                               self._ptr(self._flags), v._stream()), 'cs_cfr_train')
        self.iteration += int(iterations)
        self._host = None
        if isinstance(self.env, Env):   # the env holds the last deal at its root (every step was stepped back)
            self.env._sync_from_engine()

    @staticmethod
    def _ptr(t):
        return C.c_void_p(t.data_ptr())

    # -- the reference's dicts ------------------------------------------------------------------------------------
    def _tables(self):
        if self._host is None:
            self._host = dict(policy=self._policy.cpu().numpy(), average_policy=self._avg.cpu().numpy(),
                              regrets=self._regrets.cpu().numpy(), flags=self._flags.cpu().numpy())
        return self._host

    def _dict(self, name, bit):
        t = self._tables()
        out = {}
        for i in np.nonzero(t['flags'] & bit)[0]:
            out[infoset_obs(i).tobytes()] = t[name][i].copy()
        if name == 'policy':
            out.update(self._extra_policy)
        return out

    @property
    def policy(self):
        return self._dict('policy', 1)

    @property
    def average_policy(self):
        return self._dict('average_policy', 2)

    @property
    def regrets(self):
        return self._dict('regrets', 2)

    def regret_matching(self, obs):
        """cfr_agent.py:108-123 for one key."""
        regret = self.regrets[obs]
        positive_regret_sum = sum([r for r in regret if r > 0])
        action_probs = np.zeros(NUM_ACTIONS)
        for action in range(NUM_ACTIONS):
            action_probs[action] = (max(0.0, regret[action] / positive_regret_sum) if positive_regret_sum > 0
                                    else 1.0 / NUM_ACTIONS)
        return action_probs

    def action_probs(self, obs, legal_actions, policy):
        """cfr_agent.py:125-146. Like the reference, an unseen key gets the uniform row and is inserted into
        self.policy (whichever dict was searched)."""
        if obs not in policy.keys():
            action_probs = np.array([1.0 / NUM_ACTIONS for _ in range(NUM_ACTIONS)])
            self._insert_policy(obs, action_probs)
        else:
            action_probs = policy[obs]
        return remove_illegal(action_probs, legal_actions)

    def _insert_policy(self, obs, row):
        idx = obs_infoset(np.frombuffer(obs, dtype=np.float64)) if len(obs) == 36 * 8 else -1
        if idx < 0:
            self._extra_policy[obs] = row
            return
        self._policy[idx] = torch.as_tensor(row, dtype=torch.float64)
        self._flags[idx] |= 1
        self._host = None

    def eval_step(self, state):
        """cfr_agent.py:148-165: a draw from the average policy (global np.random, as the reference)."""
        legal = list(state['legal_actions'].keys())
        probs = self.action_probs(np.asarray(state['obs']).tobytes(), legal, self.average_policy)
        action = np.random.choice(len(probs), p=probs)
        info = {'probs': {state['raw_legal_actions'][i]: float(probs[legal[i]]) for i in range(len(legal))}}
        return action, info

    def get_state(self, player_id):
        """cfr_agent.py:167-180: (obs bytes, legal ids) of the env."""
        state = self.env.get_state(player_id)
        return state['obs'].tobytes(), list(state['legal_actions'].keys())

    # -- persistence (our own npz format; the reference pickles its dicts) ------------------------------------------
    def save(self):
        os.makedirs(self.model_path, exist_ok=True)
        t = self._tables()
        np.savez(os.path.join(self.model_path, 'cfr_tables.npz'), policy=t['policy'], average_policy=t['average_policy'],
                 regrets=t['regrets'], flags=t['flags'], iteration=np.int64(self.iteration))

    def load(self):
        path = os.path.join(self.model_path, 'cfr_tables.npz')
        if not os.path.exists(path):
            return
        d = np.load(path, allow_pickle=False)
        self._policy.copy_(torch.from_numpy(d['policy']))
        self._avg.copy_(torch.from_numpy(d['average_policy']))
        self._regrets.copy_(torch.from_numpy(d['regrets']))
        self._flags.copy_(torch.from_numpy(d['flags'].astype(np.int32)))
        self.iteration = int(d['iteration'])
        self._host = None
