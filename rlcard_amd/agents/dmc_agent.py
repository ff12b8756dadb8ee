"""DMC (Deep Monte-Carlo) on the device: the learner's side of the rollout.

* DMCNet / DMCAgent / DMCModel -- rlcard/agents/dmc_agent/model.py:21-175: the same torch module layout
  (`fc_layers` = Linear/ReLU stack, so a reference state_dict loads unchanged) and the single-state agent API
  (step / eval_step / predict) used through rlcard_amd.make(...).run().
* ActorBuffers -- rlcard/agents/dmc_agent/utils.py:49-163 (create_buffers / act / get_batch) for every env of a VecEnv
  at once: rollout trajectories go straight into per-(env, player) int8 rings in HBM (cs_dmc_fill), finished T-row
  chunks come out as learner batches [T][B][...] (cs_dmc_gather). No host round trip.
* q_values / select_actions / DMCActor -- DMCAgent.predict / step over every env's legal actions at once: the first
  Linear layer is split into W_obs . obs (one GEMM per state) + W_act . feature (fused per legal action with bias and
  ReLU in cs_dmc_layer1), the hidden layers are plain GEMMs, cs_dmc_select takes the per-state argmax (epsilon-greedy
  with Philox in place of the reference's np.random).
"""
import ctypes as C

import numpy as np
import torch
from torch import nn

from .. import _abi


def _ptr(t):
    return None if t is None else C.c_void_p(t.data_ptr())


class DMCNet(nn.Module):
    """model.py:21-43: MLP over [flatten(obs), flatten(action feature)] -> one value."""

    def __init__(self, state_shape, action_shape, mlp_layers=(512, 512, 512, 512, 512)):
        super().__init__()
        input_dim = int(np.prod(state_shape)) + int(np.prod(action_shape))
        dims = [input_dim] + list(mlp_layers)
        fc = []
        for i in range(len(dims) - 1):
            fc.append(nn.Linear(dims[i], dims[i + 1]))
            fc.append(nn.ReLU())
        fc.append(nn.Linear(dims[-1], 1))
        self.fc_layers = nn.Sequential(*fc)
        self.obs_dim = int(np.prod(state_shape))

    def forward(self, obs, actions):
        x = torch.cat((torch.flatten(obs, 1), torch.flatten(actions, 1)), dim=1)
        return self.fc_layers(x).flatten()


class DMCAgent:
    """model.py:45-123: one player's agent; predict scores every legal action of one state."""

    def __init__(self, state_shape, action_shape, mlp_layers=(512, 512, 512, 512, 512), exp_epsilon=0.01,
                 device='0'):
        self.use_raw = False
        self.device = 'cuda:' + str(device) if str(device) != 'cpu' else 'cpu'
        self.net = DMCNet(state_shape, action_shape, mlp_layers).to(self.device)
        self.exp_epsilon = exp_epsilon
        self.action_shape = action_shape

    def step(self, state):
        action_keys, values = self.predict(state)
        if self.exp_epsilon > 0 and np.random.rand() < self.exp_epsilon:
            return np.random.choice(action_keys)
        return action_keys[int(np.argmax(values))]

    def eval_step(self, state):
        action_keys, values = self.predict(state)
        action = action_keys[int(np.argmax(values))]
        info = {'values': {state['raw_legal_actions'][i]: float(values[i]) for i in range(len(action_keys))}}
        return action, info

    def predict(self, state):
        obs = np.asarray(state['obs'], dtype=np.float32)
        keys = np.array(list(state['legal_actions'].keys()))
        feats = []
        for k, f in zip(keys, state['legal_actions'].values()):
            if f is None:   # one-hot when the env has no action features
                f = np.zeros(self.action_shape[0], dtype=np.float32)
                f[k] = 1
            feats.append(np.asarray(f, dtype=np.float32))
        feats = np.stack(feats)
        obs = np.repeat(obs[None, :], len(keys), axis=0)
        with torch.no_grad():
            v = self.net(torch.from_numpy(obs).to(self.device), torch.from_numpy(feats).to(self.device))
        return keys, v.cpu().numpy()

    def forward(self, obs, actions):
        return self.net(obs, actions)

    def parameters(self):
        return self.net.parameters()

    def load_state_dict(self, state_dict):
        return self.net.load_state_dict(state_dict)

    def state_dict(self):
        return self.net.state_dict()

    def share_memory(self):
        self.net.share_memory()

    def eval(self):
        self.net.eval()

    def set_device(self, device):
        self.device = device


class DMCModel:
    """model.py:125-175: one DMCAgent per player."""

    def __init__(self, state_shape, action_shape, mlp_layers=(512, 512, 512, 512, 512), exp_epsilon=0.01, device=0):
        self.agents = [DMCAgent(state_shape[p], action_shape[p], mlp_layers, exp_epsilon, device)
                       for p in range(len(state_shape))]

    def share_memory(self):
        for a in self.agents:
            a.share_memory()

    def eval(self):
        for a in self.agents:
            a.eval()

    def parameters(self, index):
        return self.agents[index].parameters()

    def get_agent(self, index):
        return self.agents[index]

    def get_agents(self):
        return self.agents


def shapes_of(vec):
    """DMCTrainer's shapes (trainer.py:160-170): state_shape per player (doudizhu 790 / 901 / 901) and the action
    feature shape (doudizhu 54, else a one-hot of num_actions)."""
    if vec.env_id == 'doudizhu':
        return [[790], [901], [901]], [[54]] * 3
    return [[vec.obs_dim]] * vec.num_players, [[vec.num_actions]] * vec.num_players


class ActorBuffers:
    """utils.py:49-163 for every env of `vec`: T-row chunks per (env, player) in an HBM ring of `slots` chunks."""

    def __init__(self, vec, T=100, slots=4):
        self.vec, self.T, self.slots = vec, int(T), int(slots)
        self.state_shape, _ = shapes_of(vec)
        h = C.c_void_p()
        with torch.cuda.device(vec.device):
            _abi.check(_abi.lib().cs_dmc_create(vec._h, self.T, self.slots, C.byref(h)), 'cs_dmc_create')
        self._d = h
        self.feature_dim = vec.info.action_feature_dim
        self.cap = vec.num_envs * vec.num_players * self.slots
        self._ready = torch.empty(self.cap, dtype=torch.int64, device=vec.device)
        self._nready = torch.zeros(1, dtype=torch.int64, device=vec.device)

    def close(self):
        if getattr(self, '_d', None) is not None and self._d.value:
            _abi.lib().cs_dmc_destroy(self._d)
            self._d = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def fill(self, traj):
        """Append a trajectory ([T_roll][N] rows: obs, player, action, reward, done) -> the chunk ids that became
        ready (int64 tensor), in (env, player, chunk) order."""
        T = traj['player'].shape[0]
        s = _abi.TrajOut(_ptr(traj['obs']), None, _ptr(traj['player']), _ptr(traj['action']), _ptr(traj['reward']),
                         _ptr(traj['done']), None)
        with torch.cuda.device(self.vec.device):
            _abi.check(_abi.lib().cs_dmc_fill(self._d, int(T), C.byref(s), _ptr(self._ready), self.cap,
                                              _ptr(self._nready), self.vec._stream()), 'cs_dmc_fill')
        n = int(self._nready.item())
        if self.dropped():
            raise _abi.CardsimError('DMC actor buffers overflowed: a (env, player) ring of %d chunks was full, rows were '
                                    'dropped (gather the ready chunks before the next fill, or use more slots)'
                                    % self.slots)
        return self._ready[:n].clone()

    def player_of(self, chunks):
        return (chunks // self.slots) % self.vec.num_players

    def get_batch(self, player, chunks):
        """utils.py:33-46: chunks of one player -> dict(done, episode_return, target, state, action) of [T, B, ...]."""
        B, T, d = int(chunks.numel()), self.T, self.vec.device
        out = dict(done=torch.empty((T, B), dtype=torch.bool, device=d),
                   episode_return=torch.empty((T, B), dtype=torch.float32, device=d),
                   target=torch.empty((T, B), dtype=torch.float32, device=d),
                   state=torch.empty((T, B, self.state_shape[player][0]), dtype=torch.int8, device=d),
                   action=torch.empty((T, B, self.feature_dim), dtype=torch.int8, device=d))
        if B:
            ch = chunks.to(device=d, dtype=torch.int64).contiguous()
            b = _abi.DmcBatch(_ptr(out['state']), _ptr(out['action']), _ptr(out['target']), _ptr(out['done']),
                              _ptr(out['episode_return']))
            with torch.cuda.device(d):
                _abi.check(_abi.lib().cs_dmc_gather(self._d, int(player), _ptr(ch), B, C.byref(b),
                                                    self.vec._stream()), 'cs_dmc_gather')
        return out

    def dropped(self):
        v = C.c_uint32()
        _abi.check(_abi.lib().cs_dmc_status(self._d, C.byref(v)), 'cs_dmc_status')
        return bool(v.value & 1)


def q_values(vec, net, obs, state_of, ids):
    """DMCNet values of legal entries (state_of[i], ids[i]) for states obs ([S, obs_dim] uint8/int8, 0/1 values):
    the reference's predict (model.py:91-110) for every state at once. -> float32 [E]."""
    with torch.no_grad():
        return _q_values(vec, net, obs, state_of, ids)


def _q_values(vec, net, obs, state_of, ids):
    lin = [m for m in net.fc_layers if isinstance(m, nn.Linear)]
    W1, b1 = lin[0].weight, lin[0].bias
    O = net.obs_dim
    H = W1.shape[0]
    X = torch.nn.functional.linear(obs[:, :O].float(), W1[:, :O])                    # [S, H] per state
    Wa = W1[:, O:].t().contiguous()                                                 # [F, H]
    E = int(ids.numel())
    h = torch.empty((E, H), dtype=torch.float32, device=obs.device)
    if E:
        with torch.cuda.device(obs.device):
            _abi.check(_abi.lib().cs_dmc_layer1(vec._h, _ptr(X.contiguous()), _ptr(state_of), _ptr(ids), E, H,
                                                _ptr(Wa), _ptr(b1.contiguous()), _ptr(h),
                                                C.c_void_p(torch.cuda.current_stream(obs.device).cuda_stream)),
                       'cs_dmc_layer1')
    for m in list(net.fc_layers)[2:]:
        h = m(h)
    return h.flatten()


def select_actions(values, counts, offsets, ids, eps=0.0, seed=0, t=0, state_base=0):
    """Per state: argmax over its legal entries (first maximum), or with probability eps a uniform legal id."""
    S = int(counts.numel())
    out = torch.empty(S, dtype=torch.int32, device=values.device)
    if S:
        with torch.cuda.device(values.device):
            _abi.check(_abi.lib().cs_dmc_select(_ptr(values.contiguous()), _ptr(counts), _ptr(offsets), _ptr(ids), S,
                                                float(eps), int(seed) & (2 ** 64 - 1), int(t), int(state_base),
                                                _ptr(out), C.c_void_p(torch.cuda.current_stream(values.device)
                                                                      .cuda_stream)), 'cs_dmc_select')
    return out


class DMCActor:
    """utils.py:97-163 act for every env of a VecEnv: each step, every env's acting player scores its legal actions
    with its own DMCNet (q_values) and picks with select_actions; the steps land in a trajectory buffer that fills the
    ActorBuffers. A step on a finished game starts the next one (lazy auto-reset) and is not a transition (player
    255 in the trajectory)."""

    def __init__(self, vec, model, T=100, slots=None, exp_epsilon=0.01, seed=0, steps_per_fill=None):
        self.vec, self.model = vec, model
        self.steps_per_fill = int(steps_per_fill or T)
        if slots is None:   # the chunk being filled, one handed out, a fill's rows, the longest game's rows
            slots = 3 + (self.steps_per_fill + T - 1) // T
        self.buffers = ActorBuffers(vec, T, slots)
        self.eps, self.seed, self.t = float(exp_epsilon), int(seed), 0
        self.state = vec.reset()
        self.traj = vec.new_traj_out(self.steps_per_fill)
        self.nets = [a.net for a in model.get_agents()]

    def policy(self, state):
        counts, offsets, ids = self.vec.legal_lists(state['legal'])
        S = self.vec.num_envs
        state_of = torch.repeat_interleave(torch.arange(S, device=ids.device, dtype=torch.int32),
                                           counts.long(), output_size=int(ids.numel()))
        values = torch.zeros(ids.numel(), dtype=torch.float32, device=ids.device)
        pl = state['player'].long()
        ent_pl = pl[state_of.long()]
        with torch.no_grad():
            for p, net in enumerate(self.nets):
                sel = (ent_pl == p).nonzero().flatten()
                if sel.numel():
                    values[sel] = q_values(self.vec, net, state['obs'], state_of[sel].contiguous(),
                                           ids[sel].contiguous())
        return select_actions(values, counts, offsets, ids, self.eps, self.seed, self.t, self.vec.env_base)

    def act(self):
        """steps_per_fill env steps -> {player: ready chunk ids}; batches via self.buffers.get_batch."""
        tr, st = self.traj, self.state
        for k in range(self.steps_per_fill):
            acts = self.policy(st)
            done_before = st['done'].bool()
            tr['obs'][k].copy_(st['obs'])
            tr['legal'][k].copy_(st['legal'])
            tr['player'][k].copy_(torch.where(done_before, torch.full_like(st['player'], 255), st['player']))
            tr['action'][k].copy_(acts.clamp_min(0).to(tr['action'].dtype))
            st = self.vec.step(acts)
            tr['reward'][k].copy_(st['reward'])
            tr['done'][k].copy_(st['done'])
            self.t += 1
        self.state = st
        ready = self.buffers.fill(tr)
        pl = self.buffers.player_of(ready)
        return {p: ready[pl == p] for p in range(self.vec.num_players)}
