"""ctypes binding of the CPU oracle (oracle/liboracle.so). TEST INFRASTRUCTURE ONLY: the parity checker.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg import this module.
"""
import ctypes as C
import os
import subprocess

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB_PATH = os.path.join(ROOT, 'oracle', 'liboracle.so')
GOLDEN = os.path.join(ROOT, 'tests', 'golden')

GAMES = {'blackjack': 0, 'leduc-holdem': 1, 'limit-holdem': 2, 'doudizhu': 3, 'no-limit-holdem': 4}

_lib = None


def build():
    subprocess.check_call(['make', '-s', '-C', os.path.join(ROOT, 'oracle')])


class MT(C.Structure):
    _fields_ = [('key', C.c_uint32 * 624), ('pos', C.c_int32), ('ndraw', C.c_uint64), ('philox', C.c_int32),
                ('pkey', C.c_uint32 * 2)]


class Cfg(C.Structure):
    _fields_ = [('num_players', C.c_int32), ('num_decks', C.c_int32), ('chips_for_each', C.c_int32),
                ('dealer_id', C.c_int32), ('rng_mode', C.c_int32)]


class Info(C.Structure):
    _fields_ = [('obs_dim', C.c_int32), ('num_actions', C.c_int32), ('num_players', C.c_int32),
                ('legal_bytes', C.c_int32)]


def P(a):
    return a.ctypes.data_as(C.c_void_p)


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            build()
        L = C.CDLL(LIB_PATH)
        L.or_mt_seed_int.argtypes = [C.POINTER(MT), C.c_uint32]
        L.or_mt_seed_by_array.argtypes = [C.POINTER(MT), C.c_void_p, C.c_int]
        L.or_mt_next.argtypes = [C.POINTER(MT)]
        L.or_mt_next.restype = C.c_uint32
        L.or_mt_interval.argtypes = [C.POINTER(MT), C.c_uint64]
        L.or_mt_interval.restype = C.c_uint64
        L.or_philox_u32.argtypes = [C.c_uint64, C.c_uint64, C.c_uint64]
        L.or_philox_u32.restype = C.c_uint32
        L.or_policy_pick.argtypes = [C.c_uint64, C.c_uint64, C.c_uint64, C.c_void_p, C.c_int]
        L.or_game_info.argtypes = [C.c_int, C.POINTER(Cfg), C.POINTER(Info)]
        L.or_batch_create.argtypes = [C.c_int, C.c_int64, C.POINTER(Cfg)]
        L.or_batch_create.restype = C.c_void_p
        L.or_batch_destroy.argtypes = [C.c_void_p]
        L.or_batch_seed.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p]
        L.or_batch_reset.argtypes = [C.c_void_p] + [C.c_void_p] * 5
        L.or_batch_step.argtypes = [C.c_void_p] + [C.c_void_p] * 6
        L.or_batch_observe.argtypes = [C.c_void_p, C.c_int64, C.c_int, C.c_void_p, C.c_void_p]
        L.or_batch_rollout.argtypes = [C.c_void_p, C.c_int32, C.c_uint64, C.c_uint64, C.c_uint64] + [C.c_void_p] * 7
        L.or_batch_draws.argtypes = [C.c_void_p, C.c_int64]
        L.or_batch_draws.restype = C.c_uint64
        L.or_cfr_infoset.argtypes = [C.c_void_p]
        L.or_cfr_create.argtypes = [C.c_int64, C.c_void_p, C.c_void_p]
        L.or_cfr_create.restype = C.c_void_p
        L.or_cfr_destroy.argtypes = [C.c_void_p]
        L.or_cfr_train.argtypes = [C.c_void_p, C.c_int32]
        L.or_cfr_tables.argtypes = [C.c_void_p] * 5
        L.or_cfr_draws.argtypes = [C.c_void_p, C.c_int64]
        L.or_cfr_draws.restype = C.c_uint64
        L.or_holdem_rank7.argtypes = [C.c_void_p]
        L.or_holdem_rank7.restype = C.c_uint32
        L.or_ddz_set_table.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p, C.c_int, C.c_int]
        L.or_ddz_legal_kat.argtypes = [C.c_void_p, C.c_int, C.c_void_p]
        _lib = L
        load_ddz_table()
    return _lib


def load_ddz_table():
    d = np.load(os.path.join(GOLDEN, 'ddz_actions.npz'))
    names = list(d['type_names'])
    counts = np.ascontiguousarray(d['counts'], dtype=np.uint8)
    ttype = np.ascontiguousarray(d['type'], dtype=np.int16)
    weight = np.ascontiguousarray(d['weight'], dtype=np.int16)
    _lib.or_ddz_set_table(P(counts), P(ttype), P(weight), names.index('bomb'), names.index('rocket'))


class Batch:
    """Oracle batch with the C-ABI semantics; outputs as numpy arrays."""

    def __init__(self, game, n, keys, key_len, num_players=None, num_decks=1, chips_for_each=100, dealer_id=-1,
                 rng_mode=0):
        L = lib()
        self.game = GAMES[game] if isinstance(game, str) else game
        np_ = num_players if num_players is not None else {0: 1, 1: 2, 2: 2, 3: 3, 4: 2}[self.game]
        self.cfg = Cfg(np_, num_decks, chips_for_each, dealer_id, rng_mode)
        self.info = Info()
        if L.or_game_info(self.game, C.byref(self.cfg), C.byref(self.info)) != 0:
            raise ValueError('bad game config')
        self.n = int(n)
        self.h = L.or_batch_create(self.game, self.n, C.byref(self.cfg))
        keys = np.ascontiguousarray(keys, dtype=np.uint32).reshape(self.n, 2)
        key_len = np.ascontiguousarray(key_len, dtype=np.int32).reshape(self.n)
        L.or_batch_seed(self.h, P(keys), P(key_len))

    def __del__(self):
        if getattr(self, 'h', None):
            lib().or_batch_destroy(self.h)
            self.h = None

    def _out(self, lead=()):
        i = self.info
        return dict(obs=np.zeros(lead + (self.n, i.obs_dim), np.uint8),
                    legal=np.zeros(lead + (self.n, i.legal_bytes), np.uint8),
                    player=np.zeros(lead + (self.n,), np.uint8),
                    reward=np.zeros(lead + (self.n, i.num_players), np.float32),
                    done=np.zeros(lead + (self.n,), np.uint8))

    def reset(self):
        o = self._out()
        lib().or_batch_reset(self.h, P(o['obs']), P(o['legal']), P(o['player']), P(o['reward']), P(o['done']))
        return o

    def step(self, actions):
        a = np.ascontiguousarray(actions, dtype=np.int32).reshape(self.n)
        o = self._out()
        lib().or_batch_step(self.h, P(a), P(o['obs']), P(o['legal']), P(o['player']), P(o['reward']),
                            P(o['done']))
        return o

    def observe(self, env, player):
        obs = np.zeros(self.info.obs_dim, np.uint8)
        legal = np.zeros(self.info.legal_bytes, np.uint8)
        lib().or_batch_observe(self.h, env, player, P(obs), P(legal))
        return obs, legal

    def rollout(self, T, policy_seed, t0=0, env_base=0, final_obs=False):
        o = self._out((T,))
        o['action'] = np.zeros((T, self.n), np.int32)
        fo = None
        if final_obs:
            o['final_obs'] = fo = np.zeros((T, self.n, self.info.num_players, self.info.obs_dim), np.uint8)
        lib().or_batch_rollout(self.h, T, policy_seed, t0, env_base, P(o['obs']), P(o['legal']), P(o['player']),
                               P(o['action']), P(o['reward']), P(o['done']), P(fo) if fo is not None else None)
        return o

    def draws(self, env):
        return lib().or_batch_draws(self.h, env)


CFR_INFOSETS = 2700


class CFR:
    """Oracle chance-sampling CFR (oracle/or_cfr.c) over n Leduc envs; n = 1 is the reference CFRAgent."""

    def __init__(self, keys, key_len):
        keys = np.ascontiguousarray(keys, dtype=np.uint32).reshape(-1, 2)
        key_len = np.ascontiguousarray(key_len, dtype=np.int32).reshape(-1)
        self.n = len(key_len)
        self.h = lib().or_cfr_create(self.n, P(keys), P(key_len))

    def __del__(self):
        if getattr(self, 'h', None):
            lib().or_cfr_destroy(self.h)
            self.h = None

    def train(self, iterations=1):
        lib().or_cfr_train(self.h, int(iterations))

    def tables(self):
        t = dict(policy=np.zeros((CFR_INFOSETS, 4)), average_policy=np.zeros((CFR_INFOSETS, 4)),
                 regrets=np.zeros((CFR_INFOSETS, 4)), flags=np.zeros(CFR_INFOSETS, np.uint8))
        lib().or_cfr_tables(self.h, P(t['policy']), P(t['average_policy']), P(t['regrets']), P(t['flags']))
        return t

    def draws(self, env):
        return lib().or_cfr_draws(self.h, env)


def cfr_infoset(obs):
    o = np.ascontiguousarray(obs, dtype=np.uint8)
    return lib().or_cfr_infoset(P(o))
