"""Single-env compatibility layer: rlcard's Env API (rlcard/envs/env.py:3-231) over one env of the HIP engine.

An Env owns a VecEnv of size 1 on one GPU and keeps rlcard's host-side contract -- reset/step/run/get_state/
get_payoffs/is_over/get_player_id/seed/timestep/action_recorder, state dicts {'obs', 'legal_actions', 'raw_obs',
'raw_legal_actions', 'action_record'} with the reference's obs dtypes and shapes -- so code written against
rlcard.make() runs unchanged. Every game rule, deal and observation is computed by the kernels; this layer only
converts one row of the engine's outputs into the reference's Python types. Throughput belongs to VecEnv.

Per Env.step the host makes one round trip: one step kernel writes the env's outputs (reward, obs, legal bitmask,
player, done) and its packed state words (the raw_obs fields) straight into one record of mapped host memory, then
a sequence number the host spins on (cs_set_step_record, _Io); the host decodes the record.
"""
import ctypes as C
import time
from collections import OrderedDict

import numpy as np
import torch

from .. import _abi, seeding
from ..vec import VecEnv, legal_ids


_hip = None


def _hip_lib():
    global _hip
    if _hip is None:
        _hip = C.CDLL('libamdhip64.so')
        _hip.hipHostMalloc.argtypes = [C.POINTER(C.c_void_p), C.c_size_t, C.c_uint]
        _hip.hipHostGetDevicePointer.argtypes = [C.POINTER(C.c_void_p), C.c_void_p, C.c_uint]
        _hip.hipHostFree.argtypes = [C.c_void_p]
        _hip.hipStreamSynchronize.argtypes = [C.c_void_p]
    return _hip


HIP_HOST_MALLOC_MAPPED, HIP_HOST_MALLOC_COHERENT = 0x2, 0x40000000
_BYTE_IDS = [tuple(i for i in range(8) if (b >> i) & 1) for b in range(256)]   # legal bitmask byte -> ids


class _Io:
    """One env's step record in mapped (device-visible, coherent) pinned host memory, written by the step kernels
    themselves (cs_set_step_record): seq u32 | pad | state words u32 [S] (16-B aligned) | reward f32 [P] | obs u8 [O]
    | legal u8 [LB] | player u8 | done u8. Actions come from a constant device table of every action id (a step reads
    actions[0] at &table[a]). So an Env.step is one launch on the env's own stream and a spin on seq -- no stream
    synchronisation, no uploads, no copies."""

    SPIN_S = 0.002   # past this the wait falls back to hipStreamSynchronize (and reports a launch failure)

    def __init__(self, vec):
        i = vec.info
        P, S, O, LB = i.num_players, i.state_words, i.obs_dim, i.legal_bytes
        self.P, self.S, self.O, self.LB = P, S, O, LB
        self.o_words = 16
        self.o_reward = self.o_words + (4 * S + 15) // 16 * 16
        self.o_obs = self.o_reward + 4 * P
        self.o_legal = self.o_obs + O
        self.o_player = self.o_legal + LB
        self.o_done = self.o_player + 1
        total = (self.o_done + 1 + 15) // 16 * 16
        hip = _hip_lib()
        with torch.cuda.device(vec.device):
            self.stream = torch.cuda.Stream(vec.device)
            self.ids = torch.arange(i.num_actions, dtype=torch.int32, device=vec.device)
            hp, dp = C.c_void_p(), C.c_void_p()
            if hip.hipHostMalloc(C.byref(hp), total, HIP_HOST_MALLOC_MAPPED | HIP_HOST_MALLOC_COHERENT) != 0:
                raise _abi.CardsimError('hipHostMalloc of the step record failed')
            self._hp = hp
            if hip.hipHostGetDevicePointer(C.byref(dp), hp, 0) != 0:
                raise _abi.CardsimError('hipHostGetDevicePointer of the step record failed')
        self.np = np.frombuffer((C.c_uint8 * total).from_address(hp.value), dtype=np.uint8)
        self.np[:] = 0
        self.seq = self.np[:4].view(np.uint32)
        base = dp.value
        self.st = C.c_void_p(self.stream.cuda_stream)
        self.out = _abi.StepOut(C.c_void_p(base + self.o_obs), C.c_void_p(base + self.o_legal),
                                C.c_void_p(base + self.o_player), C.c_void_p(base + self.o_reward),
                                C.c_void_p(base + self.o_done))
        self.obs_out = _abi.StepOut(self.out.obs, self.out.legal, self.out.player, None, self.out.done)
        self.ids_base = self.ids.data_ptr()
        self.vec = vec   # the record stays registered on vec's handle until close()
        _abi.check(_abi.lib().cs_set_step_record(vec._h, 0, C.c_void_p(base + self.o_words), C.c_void_p(base)),
                   'cs_set_step_record')
        self.expect = 0

    def act_ptr(self, a):
        return C.c_void_p(self.ids_base + 4 * a)

    def wait(self):
        """Spin until the kernel has published this call's record (seq), else synchronise and report."""
        self.expect = (self.expect + 1) & 0xFFFFFFFF
        seq, want = self.seq, self.expect
        if seq[0] == want:
            return
        t0 = time.perf_counter()
        while seq[0] != want:
            if time.perf_counter() - t0 > self.SPIN_S:
                if _hip.hipStreamSynchronize(self.st) != 0:
                    raise _abi.CardsimError('hipStreamSynchronize failed: %s' % _abi.lib().cs_last_error().decode())
                if seq[0] != want:
                    raise _abi.CardsimError('step record not published (seq %d, expected %d)' % (seq[0], want))
                return

    def close(self):
        if getattr(self, '_hp', None) is not None and self._hp.value:
            vec = getattr(self, 'vec', None)
            if vec is not None and vec._h is not None:   # unregister first: later kernels must not write freed memory
                torch.cuda.synchronize(vec.device)
                _abi.lib().cs_set_step_record(vec._h, 0, None, None)
            _hip_lib().hipHostFree(self._hp)
            self._hp = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def record(self, with_reward=True):
        h = self.np
        out = {'obs': h[self.o_obs:self.o_obs + self.O].copy(), 'legal': h[self.o_legal:self.o_legal + self.LB].copy(),
               'player': int(h[self.o_player]), 'done': bool(h[self.o_done])}
        if with_reward:
            out['reward'] = h[self.o_reward:self.o_obs].view(np.float32).copy()
        words = h[self.o_words:self.o_words + 4 * self.S].view(np.uint32).tolist()
        return out, words


class Env(object):
    """Subclasses set name, default_game_config, actions, state_shape, action_shape and implement _obs_of /
    _raw_obs / get_payoffs (the reference's _extract_state / get_payoffs split)."""
    name = None
    default_game_config = {}
    configurable = False   # env.py:33-39: only blackjack / leduc / limit forward 'game_*' keys

    def __init__(self, config):
        self.allow_step_back = bool(config.get('allow_step_back', False))
        game_config = dict(self.default_game_config)
        if self.configurable:
            for k in config:
                if k in game_config:
                    game_config[k] = config[k]
        self.game_config = game_config
        self.action_recorder = []
        self.agents = None
        self._vec = VecEnv(self.name, 1, seeds=[0], device=config.get('device'), config=game_config)
        self.num_players = self._vec.num_players
        self.num_actions = self._vec.num_actions
        self._io = _Io(self._vec)
        self._words = None   # packed state words of the last record (raw_obs / get_perfect_information)
        self.timestep = 0
        self._last = None
        self._payoffs = None
        self._history = []   # step_back: (packed state words, last outputs, payoffs) before every step
        self.seed(config.get('seed'))

    # -- rlcard Env API ----------------------------------------------------------------------------------------
    def _call(self, kind, arg=0, with_reward=True):
        """One engine call on the env; the kernels write the record into mapped host memory (see _Io)."""
        io, h, L = self._io, self._vec._h, _abi.lib()
        if kind == 'step':
            _abi.check(L.cs_step(h, io.act_ptr(arg), C.byref(io.out), io.st), 'cs_step')
        elif kind == 'reset':
            _abi.check(L.cs_reset(h, C.byref(io.out), io.st), 'cs_reset')
        else:
            _abi.check(L.cs_observe(h, int(arg), C.byref(io.obs_out), io.st), 'cs_observe')
        io.wait()
        out, self._words = io.record(with_reward)
        return out

    def reset(self):
        self._before_deal()
        out = self._call('reset')
        self.action_recorder = []
        self._payoffs = None
        self._history = []
        self._last = out
        self._after_deal()
        return self._extract_state(out, out['player'], 'reset'), out['player']

    def step(self, action, raw_action=False):
        if self._last is None:
            raise RuntimeError('call reset() before step()')
        a = self._action_id(action) if raw_action else int(action)
        if not 0 <= a < self.num_actions:
            raise ValueError('action id %d out of range [0, %d)' % (a, self.num_actions))
        decoded = self._decode_action(a)
        if self.allow_step_back:
            self._history.append((self._state_words(), dict(self._last), self._payoffs, self._snapshot_extra()))
        self.timestep += 1
        player = self.get_player_id()
        self.action_recorder.append((player, decoded))
        was_over = bool(self._last['done'])
        before = self._state_words()
        if was_over:
            self._before_deal()
        out = self._call('step', self._action_id(decoded))
        if out['done']:
            self._payoffs = out['reward']
        self._last = out
        if was_over:        # lazy auto-reset: the engine dealt a new game instead (include/cardsim.h cs_step)
            self._payoffs = None
            self._history = []   # a new game: nothing to step back into (the host bookkeeping restarts with it)
            self._after_deal()
        else:
            self._after_step(player, decoded, before)
        return self._extract_state(out, out['player'], 'step'), out['player']

    def step_back(self):
        """env.py:88-108: restore the game as it was before the last step (the packed state words, written back
        with cs_set_env_state); False at the start of a game. Like the reference, whose history does not hold
        np_random, the env's RNG stream is not rewound -- except for Blackjack, whose history holds the dealer's
        RandomState (_snapshot_extra / _restore_extra)."""
        if not self.allow_step_back:
            raise Exception('Step back is off. To use step_back, please set allow_step_back=True in rlcard.make')
        if not self._history:
            return False
        words, last, payoffs, extra = self._history.pop()
        current = self._state_words()
        gw = self._vec.game_words
        if gw is not None:   # hold'em: the game words only; deals already drawn ahead stay queued
            words = list(words[:gw]) + self._vec.env_state_words(0)[gw:]
        words = self._step_back_words(list(words), current)
        self._vec.set_env_state_words(0, words)
        self._restore_extra(extra)
        self._words = list(words)
        self._last, self._payoffs = last, payoffs
        self._after_step_back()
        player_id = self.get_player_id()
        return self.get_state(player_id), player_id

    def set_agents(self, agents):
        self.agents = agents

    def run(self, is_training=False):
        """env.py:120-169: one game, trajectories[p] = [state, action, state, ..., final state] + payoffs."""
        trajectories = [[] for _ in range(self.num_players)]
        state, player_id = self.reset()
        trajectories[player_id].append(state)
        while not self.is_over():
            if not is_training:
                action, _ = self.agents[player_id].eval_step(state)
            else:
                action = self.agents[player_id].step(state)
            next_state, next_player_id = self.step(action, self.agents[player_id].use_raw)
            trajectories[player_id].append(action)
            state, player_id = next_state, next_player_id
            if not self.is_over():
                trajectories[player_id].append(state)
        for p in range(self.num_players):
            trajectories[p].append(self.get_state(p))
        return trajectories, self.get_payoffs()

    def is_over(self):
        return bool(self._last is not None and self._last['done'])

    def get_player_id(self):
        return int(self._last['player'])

    def get_state(self, player_id):
        return self._extract_state(self._call('observe', player_id, with_reward=False), player_id)

    def get_payoffs(self):
        r = self._payoffs if self._payoffs is not None else np.zeros(self.num_players, np.float32)
        return self._payoff_array(r)

    def get_perfect_information(self):
        raise NotImplementedError

    def get_action_feature(self, action):
        feature = np.zeros(self.num_actions, dtype=np.int8)
        feature[action] = 1
        return feature

    def seed(self, seed=None):
        """env.py:228-231 + utils/seeding.py: same seed -> same init_by_array key -> same deals."""
        s = seeding.create_seed(seed)
        self._vec.seed([s])
        self._last = None
        self._words = None
        return s

    def _sync_from_engine(self):
        """Re-read the env's current game from the engine after device-side work that moved it (cs_cfr_train leaves
        the last deal at its root, as the reference's traversal leaves its env after stepping every step back)."""
        torch.cuda.current_stream(self._vec.device).synchronize()   # device work was queued on the caller's stream
        o = self._call('observe', 0, with_reward=False)
        if o['player'] != 0:
            o = self._call('observe', o['player'], with_reward=False)
        o['reward'] = np.zeros(self.num_players, np.float32)
        self._last, self._payoffs, self._history = o, None, []

    # -- engine row -> reference types ---------------------------------------------------------------------------
    def _legal_ids(self, out):
        lg = out['legal']
        if len(lg) == 1:   # one bitmask byte (every game but doudizhu): table lookup
            return list(_BYTE_IDS[int(lg[0])])
        return legal_ids(lg)

    def _extract_state(self, out, player_id, via='get_state'):
        """via: 'reset', 'step' or 'get_state' -- the Game method whose state dict the reference's raw_obs is (their
        key orders differ for Blackjack, games/blackjack/game.py:104-117 vs 162-190)."""
        ids = self._legal_order(out)
        state = {
            'legal_actions': OrderedDict((i, self._legal_value(i)) for i in ids),
            'obs': self._obs_of(out['obs'], player_id),
            'raw_obs': self._raw_obs(player_id, ids, via),
            'raw_legal_actions': [self._raw_action(i) for i in ids],
            'action_record': self.action_recorder,
        }
        return state

    def _legal_order(self, out):
        """The legal ids in the order the reference lists them (ascending for every game but DouDizhu)."""
        return self._legal_ids(out)

    # host-side bookkeeping of raw fields the engine state does not hold (DouDizhu's trace and suit-level hands,
    # No-limit's Python / numpy integer types); `before` = the packed state words the step started from
    def _after_deal(self):
        pass

    def _after_step(self, player, decoded, before):
        pass

    def _after_step_back(self):
        pass

    # device-side parts of the step_back history beyond the state words (Blackjack: the dealer's RandomState)
    def _snapshot_extra(self):
        return None

    def _restore_extra(self, extra):
        pass

    def _before_deal(self):
        """Called before the engine deals a new game (reset, or the lazy auto-reset of a step on a finished game)."""
        pass

    def _step_back_words(self, words, current):
        """The state words step_back writes: the snapshot, amended where the reference's Game.step_back does not
        restore everything it saved (limit hold'em's raise history, no-limit's round pot)."""
        return words

    def _legal_value(self, action_id):
        return None

    def _raw_action(self, action_id):
        return self.actions[action_id]

    def _action_id(self, raw):
        if isinstance(raw, (int, np.integer)):
            return int(raw)
        return self.actions.index(raw)

    def _decode_action(self, action_id):
        return self._raw_action(action_id)

    def _obs_of(self, obs_bytes, player_id):
        return obs_bytes.astype(np.float64)

    def _raw_obs(self, player_id, legal, via):
        return None

    def _payoff_array(self, r):
        return np.asarray(r, dtype=np.float64)

    def _state_words(self):
        if self._words is None:
            self._words = self._vec.env_state_words(0)
        return self._words
