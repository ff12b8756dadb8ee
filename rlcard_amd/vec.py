"""Batched lockstep envs on one GPU: the hot path behind rlcard_amd.make() and bench.py.

A VecEnv holds `num_envs` independent games of one kind in HBM (one C-ABI handle, include/cardsim.h). Outputs are
torch tensors on the env's device, written by the HIP kernels on the current torch stream:

  obs    uint8   [N, obs_dim]      Env._extract_state(...)['obs'] of the current player (0/1 values; blackjack scores)
  legal  uint8   [N, legal_bytes]  legal action ids as a little-endian bitmask (see legal_mask())
  player uint8   [N]               Env.get_player_id()
  reward float32 [N, num_players]  Env.get_payoffs() on the step that ends a game, else 0
  done   uint8   [N]               Env.is_over()

Env i is seeded with seeds[i] (default: seed + env_base + i) exactly as rlcard.make(..., config={'seed': s}) seeds
its numpy RandomState, so env i replays the reference's deals for that seed.
"""
import ctypes as C
import time

import numpy as np
import torch

from . import _abi
from .seeding import seed_keys

__all__ = ['VecEnv', 'legal_mask', 'legal_ids']


def legal_mask(legal_bytes, num_actions):
    """uint8 [..., legal_bytes] bitmask -> bool [..., num_actions]."""
    bits = torch.arange(8, device=legal_bytes.device, dtype=torch.uint8)
    m = (legal_bytes.unsqueeze(-1) >> bits) & 1
    return m.reshape(*legal_bytes.shape[:-1], -1)[..., :num_actions].bool()


def legal_ids(legal_row):
    """One env's bitmask (1-d uint8, any device) -> sorted list of legal action ids."""
    b = np.unpackbits(np.asarray(legal_row.cpu() if torch.is_tensor(legal_row) else legal_row, dtype=np.uint8),
                      bitorder='little')
    return [int(i) for i in np.nonzero(b)[0]]


def _ptr(t):
    return None if t is None else C.c_void_p(t.data_ptr())


class VecEnv:
    def __init__(self, env_id, num_envs, seed=0, seeds=None, device=None, config=None, env_base=0):
        config = dict(config or {})
        self.env_id = env_id
        if env_id not in _abi.GAME_IDS:
            raise ValueError('Cannot find env_id: {}'.format(env_id))
        self.game = _abi.GAME_IDS[env_id]
        self.num_envs = int(num_envs)
        self.env_base = int(env_base)
        if device is None:
            device = torch.cuda.current_device() if torch.cuda.is_available() else 0
        self.device = torch.device('cuda', device) if isinstance(device, int) else torch.device(device)
        if self.device.type != 'cuda':
            raise _abi.CardsimError('VecEnv runs on the GPU only (got device %s)' % self.device)
        np_ = int(config.get('game_num_players', 0))
        nd = int(config.get('game_num_decks', -1))
        chips = int(config.get('chips_for_each', 0))
        self.rng_mode = config.get('rng_mode', 'mt19937')   # 'philox': fast, not the reference's deals
        self.info, self.cfg = _abi.game_info(self.game, np_, nd, chips, config.get('dealer_id'), self.rng_mode)
        self.obs_dim = self.info.obs_dim
        self.num_actions = self.info.num_actions
        self.num_players = self.info.num_players
        self.legal_bytes = self.info.legal_bytes
        self.action_dtype = torch.uint8 if self.info.action_bytes == 1 else torch.int16
        L = _abi.lib()
        h = C.c_void_p()
        _abi.check(L.cs_create(C.byref(h), self.game, self.num_envs, self.device.index or 0, C.byref(self.cfg)),
                   'cs_create')
        self._h = h
        if seeds is None:
            seeds = range(int(seed) + self.env_base, int(seed) + self.env_base + self.num_envs)
        self.seed(seeds)

    # -- lifetime ----------------------------------------------------------------------------------------------
    def close(self):
        if getattr(self, '_h', None) is not None and self._h.value:
            _abi.lib().cs_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def _stream(self):
        return C.c_void_p(torch.cuda.current_stream(self.device).cuda_stream)

    # -- API -----------------------------------------------------------------------------------------------------
    def seed(self, seeds, first_env=0):
        keys, lens = seed_keys(seeds)
        n = len(lens)
        with torch.cuda.device(self.device):
            _abi.check(_abi.lib().cs_seed(self._h, keys.ctypes.data_as(C.c_void_p), lens.ctypes.data_as(C.c_void_p),
                                          first_env, n, self._stream()), 'cs_seed')

    def new_step_out(self, lead=()):
        n, d = self.num_envs, self.device
        return dict(obs=torch.empty(lead + (n, self.obs_dim), dtype=torch.uint8, device=d),
                    legal=torch.empty(lead + (n, self.legal_bytes), dtype=torch.uint8, device=d),
                    player=torch.empty(lead + (n,), dtype=torch.uint8, device=d),
                    reward=torch.empty(lead + (n, self.num_players), dtype=torch.float32, device=d),
                    done=torch.empty(lead + (n,), dtype=torch.uint8, device=d))

    @staticmethod
    def _step_struct(o):
        return _abi.StepOut(_ptr(o.get('obs')), _ptr(o.get('legal')), _ptr(o.get('player')), _ptr(o.get('reward')),
                            _ptr(o.get('done')))

    def reset(self, out=None):
        o = out if out is not None else self.new_step_out()
        with torch.cuda.device(self.device):
            _abi.check(_abi.lib().cs_reset(self._h, C.byref(self._step_struct(o)), self._stream()), 'cs_reset')
        return o

    def step(self, actions, out=None):
        a = torch.as_tensor(actions, device=self.device).to(torch.int32).contiguous()
        if a.numel() != self.num_envs:
            raise ValueError('expected %d actions, got %d' % (self.num_envs, a.numel()))
        o = out if out is not None else self.new_step_out()
        with torch.cuda.device(self.device):
            _abi.check(_abi.lib().cs_step(self._h, _ptr(a), C.byref(self._step_struct(o)), self._stream()),
                       'cs_step')
        return o

    def observe(self, player, out=None):
        o = out if out is not None else self.new_step_out()
        o = {k: o[k] for k in ('obs', 'legal', 'player', 'done')}
        with torch.cuda.device(self.device):
            _abi.check(_abi.lib().cs_observe(self._h, int(player), C.byref(self._step_struct(o)), self._stream()),
                       'cs_observe')
        return o

    # trajectory candidates new_traj_out allocates and ranks by default (placement): where a trajectory lands
    # in HBM sets how fast the rollout can write it -- one allocation in three or so takes the rollout's writes 15-25 %
    # slower, which the write-only probe tells apart, and within the fast class a few % more that only the rollout
    # itself shows
    PLACEMENT_CANDIDATES = 4
    FAST_CLASS = 0.93        # a candidate probing at >= this fraction of the best rate seen for its shape is "fast"
    _probe_best = {}         # (game, envs, T, final_obs) -> best probe rate (B/ms) seen in this process

    def traj_bytes(self, T, final_obs=False):
        """HBM bytes of one trajectory [T, N, ...] (new_traj_out's tensors)."""
        i = self.info
        per = i.obs_dim + i.legal_bytes + 1 + i.action_bytes + 4 * i.num_players + 1
        if final_obs:
            per += i.num_players * i.obs_dim
        return int(T) * self.num_envs * per

    def state_bytes(self):
        """bytes of the envs' whole engine state (include/cardsim.h cs_state_bytes), 0 on a library without it"""
        L = _abi.lib()
        if not hasattr(L, 'cs_state_bytes'):
            return 0
        n = C.c_int64()
        _abi.check(L.cs_state_bytes(self._h, C.byref(n)), 'cs_state_bytes')
        return n.value

    def save_state(self, buf=None):
        """the envs' whole engine state into a device buffer (cs_state_save; async on the env's stream) -> the buffer"""
        if buf is None:
            buf = torch.empty(self.state_bytes(), dtype=torch.uint8, device=self.device)
        with torch.cuda.device(self.device):
            _abi.check(_abi.lib().cs_state_save(self._h, _ptr(buf), self._stream()), 'cs_state_save')
        return buf

    def load_state(self, buf):
        """the envs' whole engine state back from save_state's buffer (cs_state_load): rollouts, steps and resets
        since the save are undone"""
        with torch.cuda.device(self.device):
            _abi.check(_abi.lib().cs_state_load(self._h, _ptr(buf), self._stream()), 'cs_state_load')

    def new_traj_out(self, T, final_obs=False, select=None, rank='rollout'):
        """Trajectory buffers [T, N, ...] for rollout(). The placement is chosen: up to `select` candidates (default
        PLACEMENT_CANDIDATES, fewer when free device memory does not hold them all at once) are allocated side by
        side and each is timed with the placement probe (probe_traj: the rollout's writes, zeros, no env state
        touched). rank='rollout' (the default): the candidates probing within FAST_CLASS of the best are then timed by
        one rollout launch each (after one untimed launch) -- the envs' state saved before and loaded after
        (save_state / load_state), so the envs end where they were -- and the fastest is kept; rank='probe': the fastest probe is kept, and on the
        default path the draw stops early at a candidate probing in the fast class of the best rate this process has
        seen for the shape. The others go back to torch's caching allocator. select=1: the first allocation,
        untimed. Left in self: placement_probe_ms / placement_trial_ms (per candidate, None where not timed) and
        placement_select_ms (the time the choice took)."""
        def one():
            o = self.new_step_out((T,))
            o['action'] = torch.empty((T, self.num_envs), dtype=self.action_dtype, device=self.device)
            if final_obs:   # every player's observation where a game ended (Env.run's final states)
                o['final_obs'] = torch.zeros((T, self.num_envs, self.num_players, self.obs_dim), dtype=torch.uint8,
                                             device=self.device)
            return o
        if rank not in ('rollout', 'probe'):
            raise ValueError("rank must be 'rollout' or 'probe'")
        k = self.PLACEMENT_CANDIDATES if select is None else int(select)
        nbytes = self.traj_bytes(T, final_obs)
        sbytes = self.state_bytes() if rank == 'rollout' else 0
        if rank == 'rollout' and sbytes == 0:
            rank = 'probe'   # (a library without cs_state_*)
        if k > 1:
            free, _ = torch.cuda.mem_get_info(self.device)
            k = min(k, (int(0.9 * free) - sbytes) // max(1, nbytes))
        self.placement_probe_ms = None
        self.placement_trial_ms = None
        self.placement_select_ms = 0.0
        if k <= 1:
            return one()
        t0 = time.perf_counter()
        key = (self.game, self.num_envs, int(T), bool(final_obs))
        ref = VecEnv._probe_best.get(key, 0.0)   # from earlier choices in this process (the first draws all k)
        cands, times = [], []
        for i in range(k):   # candidates alive together, so each is a fresh placement
            c = one()
            cands.append(c)
            times.append(min(self.probe_traj(c, T) for _ in range(2)))
            if rank == 'probe' and select is None and ref > 0 and nbytes / times[-1] >= self.FAST_CLASS * ref:
                break   # (default probe path: a candidate in the shape's fast class ends the draw)
        VecEnv._probe_best[key] = max(ref, nbytes / min(times))
        self.placement_probe_ms = times
        best, self.placement_trial_ms = self.rank_placements(cands, T, times, rank)
        self.placement_select_ms = (time.perf_counter() - t0) * 1e3
        return cands[best]

    def rank_placements(self, cands, T, probe_ms, rank='rollout'):
        """new_traj_out's choice among candidate trajectories with their probe times: rank='probe' the fastest
        probe; rank='rollout' the candidates probing within FAST_CLASS of the best, timed by one rollout launch each
        after one untimed launch, the envs' state saved before and loaded after. -> (index, trial ms per candidate
        or None)"""
        if rank == 'probe' or len(cands) == 1:
            return min(range(len(cands)), key=lambda i: probe_ms[i]), None
        fast = [i for i in range(len(cands)) if min(probe_ms) >= self.FAST_CLASS * probe_ms[i]]
        trial = [None] * len(cands)
        if len(fast) == 1:
            return fast[0], trial
        # (final_obs left out: the caller's rollouts only write its rows where a game ends, the others stay zero)
        main = [{k: x for k, x in c.items() if k != 'final_obs'} for c in cands]
        saved = self.save_state()
        self.rollout(T, out=main[fast[0]])
        for i in fast:
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            with torch.cuda.device(self.device):
                e0.record()
                self.rollout(T, out=main[i])
                e1.record()
                e1.synchronize()
            trial[i] = e0.elapsed_time(e1)
        self.load_state(saved)
        torch.cuda.current_stream(self.device).synchronize()
        return min(fast, key=lambda i: trial[i]), trial

    def probe_traj(self, traj, T=None):
        """ms of one placement probe (include/cardsim.h cs_traj_probe: the rollout's writes, zeros, no state change)
        over the trajectory `traj`, timed with events on the env's stream."""
        T = int(T if T is not None else traj['player'].shape[0])
        s = _abi.TrajOut(_ptr(traj['obs']), _ptr(traj['legal']), _ptr(traj['player']), _ptr(traj['action']),
                         _ptr(traj['reward']), _ptr(traj['done']), None)
        with torch.cuda.device(self.device):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            _abi.check(_abi.lib().cs_traj_probe(self._h, T, C.byref(s), self._stream()), 'cs_traj_probe')
            e1.record()
            e1.synchronize()
        return e0.elapsed_time(e1)

    def rollout(self, T, policy_seed=0, t0=0, out=None, final_obs=False):
        """T lockstep steps of the uniform-random legal policy, auto-reset; -> trajectory dict of [T, N, ...]
        (+ 'final_obs' [T, N, P, obs_dim] where a game ended, when asked for or present in `out`). Without `out`,
        the trajectory comes from new_traj_out (placement chosen); pass `out` to reuse one across launches."""
        o = out if out is not None else self.new_traj_out(T, final_obs)
        s = _abi.TrajOut(_ptr(o['obs']), _ptr(o['legal']), _ptr(o['player']), _ptr(o['action']),
                         _ptr(o['reward']), _ptr(o['done']), _ptr(o.get('final_obs')))
        with torch.cuda.device(self.device):
            _abi.check(_abi.lib().cs_rollout(self._h, int(T), int(policy_seed) & (2 ** 64 - 1), int(t0),
                                             self.env_base, C.byref(s), self._stream()), 'cs_rollout')
        return o

    # -- after the rollout ----------------------------------------------------------------------------
    def transitions(self, traj):
        """rlcard's reorganize + DMC return target of a rollout trajectory (include/cardsim.h cs_transitions):
        dict of [T, N] tensors next_t, end_t (int32), reward, ret (float32), done (uint8)."""
        T = traj['player'].shape[0]
        d = self.device
        o = dict(next_t=torch.empty((T, self.num_envs), dtype=torch.int32, device=d),
                 end_t=torch.empty((T, self.num_envs), dtype=torch.int32, device=d),
                 reward=torch.empty((T, self.num_envs), dtype=torch.float32, device=d),
                 done=torch.empty((T, self.num_envs), dtype=torch.uint8, device=d),
                 ret=torch.empty((T, self.num_envs), dtype=torch.float32, device=d))
        tr = _abi.TrajOut(None, None, _ptr(traj['player']), None, _ptr(traj['reward']), _ptr(traj['done']), None)
        so = _abi.TransOut(*(_ptr(o[k]) for k in ('next_t', 'end_t', 'reward', 'done', 'ret')))
        with torch.cuda.device(self.device):
            _abi.check(_abi.lib().cs_transitions(self._h, int(T), C.byref(tr), C.byref(so), self._stream()),
                       'cs_transitions')
        return o

    def legal_lists(self, legal):
        """Bitmask rows [..., legal_bytes] -> (counts int32 [R], offsets int64 [R+1], ids int32 [total]): every row's
        legal action ids, ascending (the keys of state['legal_actions'])."""
        rows = legal.reshape(-1, self.legal_bytes).contiguous()
        R = rows.shape[0]
        counts = torch.empty(R, dtype=torch.int32, device=self.device)
        offsets = torch.empty(R + 1, dtype=torch.int64, device=self.device)
        L, st = _abi.lib(), self._stream()
        with torch.cuda.device(self.device):
            _abi.check(L.cs_legal_lists(self._h, _ptr(rows), R, _ptr(counts), _ptr(offsets), None, st), 'cs_legal_lists')
            total = int(offsets[-1].item())
            ids = torch.empty(max(total, 1), dtype=torch.int32, device=self.device)
            _abi.check(L.cs_legal_lists(self._h, _ptr(rows), R, _ptr(counts), _ptr(offsets), _ptr(ids), st),
                       'cs_legal_lists')
        return counts, offsets, ids[:total]

    def action_features(self, ids):
        """Env.get_action_feature for a tensor of action ids -> uint8 [len(ids), action_feature_dim]."""
        ids = torch.as_tensor(ids, device=self.device).to(torch.int32).contiguous().reshape(-1)
        out = torch.empty((ids.numel(), self.info.action_feature_dim), dtype=torch.uint8, device=self.device)
        if ids.numel():
            with torch.cuda.device(self.device):
                _abi.check(_abi.lib().cs_action_features(self._h, _ptr(ids), ids.numel(), _ptr(out), self._stream()),
                           'cs_action_features')
        return out

    # -- introspection (synchronous) ------------------------------------------------------------------------------
    def env_state_words(self, env):
        buf = (C.c_uint32 * self.info.state_words)()
        _abi.check(_abi.lib().cs_get_env_state(self._h, int(env), buf, self.info.state_words), 'cs_get_env_state')
        return list(buf)

    def set_env_state_words(self, env, words):
        buf = (C.c_uint32 * self.info.state_words)(*[int(w) & 0xFFFFFFFF for w in words])
        _abi.check(_abi.lib().cs_set_env_state(self._h, int(env), buf, self.info.state_words), 'cs_set_env_state')

    @property
    def rng_period(self):
        """Draws after which the stream position wraps (cs_game_info.rng_period): the byte ring of the lane-per-env
        games holds RING_SLOTS_HOST blocks (rlcard_amd/csrc/cs_ring.h), doudizhu's word layout 2."""
        return int(self.info.rng_period)

    def _rng_geometry(self):
        """'words': doudizhu's two-block word window, or the Blackjack shoe's word stream (rng_period 624: one twist
        per 624 draws); 'ring': the byte ring of the other lane-per-env games (rng_period = RING_SLOTS_HOST x 624)."""
        if self.env_id == 'doudizhu':
            return 'ddz'
        return 'words' if self.rng_period == 624 else 'ring'

    @property
    def rng_first_refill(self):
        """Draws before the first refill, worst case over the envs (rng_first_refill_of): the ring games' seeding
        generates 1 + e % (SLOTS - 1) ring blocks for the handle-local env e (cs_ring.h seed_blocks) and a refill runs
        once the stream is inside the latest, so env e first refills after (e % (SLOTS - 1)) x 624 draws, at most
        (SLOTS - 2) x 624; doudizhu twists its next word block 624 draws in; the shoe's word stream twists at once."""
        g = self._rng_geometry()
        return {'ddz': 624, 'words': 0}.get(g, self.rng_period - 2 * 624)

    def rng_first_refill_of(self, env):
        """Draws before env `env`'s first refill. `env` is the handle-local index (0..num_envs-1): cs_seed's
        seed_blocks counts envs of the handle, not global ids, so shards of any env_base agree."""
        g = self._rng_geometry()
        if g == 'ddz':
            return 624
        if g == 'words':
            return 0
        return (int(env) % (self.rng_period // 624 - 1)) * 624

    @property
    def rng_per_refill(self):
        """Draws between two refills: SLOTS - 1 blocks per ring refill; doudizhu and the shoe's words one block."""
        return self.rng_period - 624 if self._rng_geometry() == 'ring' else 624

    # heads-up hold'em games keep a deal queue after their 4 game words (rlcard_amd/csrc/cs_limit.h): deals drawn
    # ahead. 3..6-player hold'em has none (its judge may draw from the stream at a game's end, cs_holdem_n.h).
    @property
    def game_words(self):
        """Packed game words before the deal queue (cs_game_info.game_words), None when the game has no queue."""
        return self.info.game_words if self.info.deal_queue_depth > 0 else None

    def game_state_words(self, env):
        """The packed game words of env `env` (without the hold'em deal queue)."""
        return self.env_state_words(env)[:self.info.game_words]

    def rng_position(self, env):
        """Draws consumed by env `env`, modulo rng_period. Deals already drawn into a hold'em env's deal queue
        do not count: they belong to the games after the current one (queue layout: include/cardsim.h,
        cs_get_env_state)."""
        v = C.c_uint32()
        _abi.check(_abi.lib().cs_get_rng_ctl(self._h, int(env), C.byref(v)), 'cs_get_rng_ctl')
        pos = v.value & (0x7FF if self.env_id == 'doudizhu' else 0x3FFF)   # cs_ring.h ctl layout
        cap = self.info.deal_queue_depth
        if cap > 0:
            gw = self.info.game_words
            w = self.env_state_words(env)
            cb = cap.bit_length()                         # header: count:cb, head:cb-1, 2 dealer bits, draws[8:7]
            xb = 2 * cb - 1
            hdr = w[gw]
            for k in range(hdr & ((1 << cb) - 1)):
                slot = (((hdr >> cb) & (cap - 1)) + k) % cap
                pos -= ((w[gw + 1 + 2 * slot] >> 25) & 127) | ((hdr >> (xb + 2 + 2 * slot)) & 3) << 7
        return pos % self.rng_period

    def set_kernel_flags(self, flags):
        _abi.check(_abi.lib().cs_debug_set_kernel_flags(self._h, int(flags)), 'cs_debug_set_kernel_flags')

    def set_serial_refill(self, enable):
        _abi.check(_abi.lib().cs_debug_set_serial_refill(self._h, 1 if enable else 0), 'cs_debug_set_serial_refill')
