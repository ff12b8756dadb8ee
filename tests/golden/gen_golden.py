#!/usr/bin/env python3
"""Generate the golden fixtures under tests/golden/ from the REFERENCE (pmcgannon22/rlcard).

Test infrastructure only. This script runs in the build container, where /root/reference exists; it never runs on
the GPU box and nothing in the product imports it. It copies the reference package into a writable temporary
directory (``rlcard/games/doudizhu/utils.py:14-19`` extracts ``jsondata.zip`` into the package dir on first import),
stubs ``termcolor`` (imported eagerly via ``rlcard/envs/__init__.py`` -> uno) and ``typing.Self`` (Python >= 3.11,
imported by the fork's scout game), then drives the reference ``Env`` objects and records inputs and outputs as
plain numpy arrays (.npz, loaded with allow_pickle=False).

Fixtures written:
  mt19937.npz      seed -> init_by_array key (rlcard/utils/seeding.py:33-113), first raw u32 outputs,
                   shuffle / randint KATs of numpy's legacy RandomState (the RNG behind every deal).
  leduc.npz        per-seed game streams: reset/step events with the action id fed in (including illegal ids,
                   to pin _decode_action's fallback), obs, legal-action bitmask, next player, done, payoffs,
                   and the final obs of every player (Env.run appends them, rlcard/envs/env.py:161-164).
  limit.npz        same for limit-holdem (pins the stale raise_nums quirk of limitholdem/game.py:98/:101).
  nolimit.npz      same for no-limit-holdem under four configs (chips_for_each / dealer_id per env: env_chips,
                   env_dealer; -1 = dealer drawn by the game).
  blackjack.npz    same for blackjack (+ the config-1 run_random.py trajectory: env seed 42, np.random.seed(42)).
  doudizhu.npz     same for doudizhu (legal ids as CSR, obs padded to 901).
  leduc_np.npz / limit_np.npz / nolimit_np.npz   the same streams with game_num_players 3..10 (env_np per env;
                   no-limit also short stacks for side pots). Leduc's obs raises IndexError in the reference when
                   the others' chips pass slot 35 (envs/leducholdem.py:64): such events are recorded with obs_len -1
                   (obs undefined there) and the game continues through Game.step, as Env.step does before it fails.
  cfr.npz          CFRAgent tables (policy, average_policy, regrets; keys = obs) after K train() iterations.
  holdem_eval.npz  compare_hands winner KATs on random and category-dense 7-card deals (limitholdem/utils.py).
  holdem_ref_kats.npz  the reference's own compare_hands known answers (tests/utils/test_holdem_utils.py), recorded.
  ddz_judger.npz   (hand, previous play) -> legal id sets from Judger / get_gt_cards (doudizhu/judger.py, utils.py),
                   plus the reference test's full-deck case (tests/games/test_doudizhu_judger.py:146-156).
  pettingzoo.json  rlcard/utils/pettingzoo_utils.py and RandomAgentPettingZoo over tests/fake_aec.py (episodes,
                   reorganized transitions, tournament means, wrap_state); JSON because the records are ragged.

Usage:  python tests/golden/gen_golden.py [--only NAME ...]
"""
import argparse
import hashlib
import json
import os
import shutil
import sys

import numpy as np

REF = '/root/reference'
WORK = '/tmp/rlcard_amd_golden_ref'
OUT = os.path.dirname(os.path.abspath(__file__))


def setup_reference():
    if not os.path.isdir(os.path.join(REF, 'rlcard')):
        sys.exit('reference not found at %s (this script only runs in the build container)' % REF)
    if os.path.isdir(WORK):
        shutil.rmtree(WORK)
    os.makedirs(os.path.join(WORK, 'stubs'))
    shutil.copytree(os.path.join(REF, 'rlcard'), os.path.join(WORK, 'rlcard'))
    with open(os.path.join(WORK, 'stubs', 'termcolor.py'), 'w') as f:
        f.write('def colored(text, *a, **k):\n    return text\n\ndef cprint(text, *a, **k):\n    print(text)\n')
    import typing
    if not hasattr(typing, 'Self'):
        typing.Self = typing.Any
    sys.path.insert(0, os.path.join(WORK, 'stubs'))
    sys.path.insert(0, WORK)
    sys.path.insert(0, os.path.dirname(OUT))   # tests/ (rawcanon)
    sys.dont_write_bytecode = True


def packbits(ids, num_actions):
    m = np.zeros(num_actions, dtype=np.uint8)
    m[list(ids)] = 1
    return np.packbits(m, bitorder='little')


# --------------------------------------------------------------------------------------------------------------
# MT19937 / seeding
# --------------------------------------------------------------------------------------------------------------
def gen_mt():
    from rlcard.utils import seeding
    seeds = [0, 1, 2, 7, 42, 43, 12941, 123456789, 2 ** 32 - 1, 2 ** 32, 2 ** 32 + 7, 2 ** 63 + 5, 2 ** 64 - 1,
             2 ** 64 + 3]
    keys = np.zeros((len(seeds), 2), dtype=np.uint32)
    key_len = np.zeros(len(seeds), dtype=np.int32)
    raw = np.zeros((len(seeds), 2000), dtype=np.uint32)
    for i, s in enumerate(seeds):
        k = seeding._int_list_from_bigint(seeding.hash_seed(seeding.create_seed(s)))
        assert 1 <= len(k) <= 2
        keys[i, :len(k)] = k
        key_len[i] = len(k)
        rng, _ = seeding.np_random(s)
        raw[i] = rng.randint(0, 2 ** 32, size=2000, dtype=np.uint32)
    # shuffles (Fisher-Yates with masked rejection) and bounded ints (randint / choice) after a fresh seed
    shuf_n = [2, 3, 6, 52, 54, 104]
    shuf = np.full((len(seeds), len(shuf_n), 104), -1, dtype=np.int16)
    bounded = np.zeros((len(seeds), 64), dtype=np.int64)
    bounded_hi = np.array([1, 2, 3, 5, 6, 7, 17, 52, 51, 100, 1000, 27471, 2, 2, 4, 9] * 4, dtype=np.int64)
    for i, s in enumerate(seeds):
        rng, _ = seeding.np_random(s)
        for j, n in enumerate(shuf_n):
            x = list(range(n))
            rng.shuffle(x)
            shuf[i, j, :n] = x
        for j, hi in enumerate(bounded_hi):
            if j % 2:
                bounded[i, j] = rng.randint(0, hi)
            else:
                bounded[i, j] = rng.choice(hi)
    # the canonical mt19937ar.c vector: init_by_array({0x123,0x234,0x345,0x456}) -> 1067595299 955945823 ...
    r = np.random.RandomState()
    r.seed([0x123, 0x234, 0x345, 0x456])
    canon = r.randint(0, 2 ** 32, size=1000, dtype=np.uint32)
    # legacy integer seeding (np.random.seed(int) -> init_genrand), used by the global agent RNG of config 1
    r = np.random.RandomState(42)
    genrand42 = r.randint(0, 2 ** 32, size=1000, dtype=np.uint32)
    np.savez_compressed(os.path.join(OUT, 'mt19937.npz'),
                        seeds=np.array([str(s) for s in seeds]), keys=keys, key_len=key_len, raw=raw,
                        shuf_n=np.array(shuf_n, dtype=np.int32), shuf=shuf, bounded_hi=bounded_hi, bounded=bounded,
                        canon_key=np.array([0x123, 0x234, 0x345, 0x456], dtype=np.uint32), canon=canon,
                        genrand42=genrand42)
    print('mt19937.npz: %d seeds' % len(seeds))


# --------------------------------------------------------------------------------------------------------------
# Game streams
# --------------------------------------------------------------------------------------------------------------
class Stream:
    """Flat per-event record of a reference Env driven by a fixed action stream."""

    def __init__(self, obs_dim, num_actions, num_players, csr_legal=False):
        self.O, self.A, self.P, self.csr = obs_dim, num_actions, num_players, csr_legal
        self.ev = {k: [] for k in ('env', 'game', 'kind', 'act', 'player', 'done', 'obs_len')}
        self.obs, self.legal, self.payoff = [], [], []
        self.legal_ids, self.legal_ptr = [], [0]
        self.fin_game, self.fin_obs, self.fin_obs_len, self.fin_legal_n = [], [], [], []

    def obs_row(self, obs):
        o = np.zeros(self.O, dtype=np.uint8)
        ob = np.asarray(obs)
        assert ob.ndim == 1 and ob.size <= self.O, ob.shape
        assert np.all((ob >= 0) & (ob <= 255)) and np.all(ob == np.round(ob)), ob
        o[:ob.size] = ob.astype(np.int64)
        return o, ob.size

    def add(self, env_i, game_i, kind, act, state, player, done, payoffs, obs_ok=True):
        o, n = self.obs_row(state['obs'])
        if not obs_ok:
            o, n = np.zeros(self.O, dtype=np.uint8), -1
        self.ev['env'].append(env_i)
        self.ev['game'].append(game_i)
        self.ev['kind'].append(kind)
        self.ev['act'].append(act)
        self.ev['player'].append(player)
        self.ev['done'].append(int(done))
        self.ev['obs_len'].append(n)
        self.obs.append(o)
        ids = sorted(state['legal_actions'].keys())
        if self.csr:
            self.legal_ids.extend(ids)
            self.legal_ptr.append(len(self.legal_ids))
        else:
            self.legal.append(packbits(ids, self.A))
        p = np.zeros(self.P, dtype=np.float64)
        if done:
            p[:len(payoffs)] = payoffs
        self.payoff.append(p)

    def add_final(self, game_i, states, oks=None):
        for k, s in enumerate(states):
            o, n = self.obs_row(s['obs'])
            if oks is not None and not oks[k]:
                o, n = np.zeros(self.O, dtype=np.uint8), -1
            self.fin_game.append(game_i)
            self.fin_obs.append(o)
            self.fin_obs_len.append(n)
            self.fin_legal_n.append(len(s['legal_actions']))

    def save(self, path, seeds, **extra):
        d = {('ev_' + k): np.array(v, dtype=np.int32) for k, v in self.ev.items()}
        d['ev_obs'] = np.stack(self.obs)
        d['ev_payoff'] = np.stack(self.payoff)
        if self.csr:
            d['ev_legal_ids'] = np.array(self.legal_ids, dtype=np.int32)
            d['ev_legal_ptr'] = np.array(self.legal_ptr, dtype=np.int64)
        else:
            d['ev_legal'] = np.stack(self.legal)
        d['fin_game'] = np.array(self.fin_game, dtype=np.int32)
        d['fin_obs'] = np.stack(self.fin_obs)
        d['fin_obs_len'] = np.array(self.fin_obs_len, dtype=np.int32)
        d['fin_legal_n'] = np.array(self.fin_legal_n, dtype=np.int32)
        d['seeds'] = np.array(seeds, dtype=np.int64)
        d.update(extra)
        np.savez_compressed(path, **d)


def drive(env_id, config, seeds, games, stream, pick, extra_keys=()):
    """For each seed: make the env once (its RNG stream continues across resets, as in the reference), then play
    `games` games, choosing each action with pick(rng, state, env). config: one dict, or one per seed."""
    import random
    import rlcard
    game_counter = 0
    for ei, seed in enumerate(seeds):
        cfg = dict(config[ei] if isinstance(config, (list, tuple)) else config)
        cfg['seed'] = int(seed)
        env = rlcard.make(env_id, config=cfg)
        rng = random.Random(1000003 * (ei + 1) + int(seed))
        for g in range(games):
            state, player = env.reset()
            stream.add(ei, game_counter, 0, -1, state, player, env.is_over(), None)
            nsteps = 0
            while not env.is_over():
                a = pick(rng, state, env)
                state, player = env.step(a)
                done = env.is_over()
                stream.add(ei, game_counter, 1, a, state, player, done, env.get_payoffs() if done else None)
                nsteps += 1
                assert nsteps < 10000
            stream.add_final(game_counter, [env.get_state(p) for p in range(env.num_players)])
            game_counter += 1


def drive_np(env_id, cfgs, seeds, games, stream):
    """drive() for N-player hold'em: Env.step (env.py:65-86) spelled out so that a failing _extract_state (Leduc's
    IndexError) leaves the event recorded with obs_len -1 and the game going. Legal actions are read from the game."""
    import random
    import rlcard
    game_counter = 0
    for ei, seed in enumerate(seeds):
        cfg = dict(cfgs[ei])
        cfg['seed'] = int(seed)
        env = rlcard.make(env_id, config=cfg)
        rng = random.Random(7919 * (ei + 1) + int(seed))

        def legal_ids():
            return sorted(env.actions.index(a) if isinstance(env.actions, list) else int(a.value)
                          for a in env.game.get_legal_actions())

        def extract(st):
            try:
                return env._extract_state(st), True
            except IndexError:
                return {'obs': np.zeros(stream.O), 'legal_actions': {i: None for i in legal_ids()}}, False

        for g in range(games):
            st, player = env.game.init_game()
            env.action_recorder = []
            state, ok = extract(st)
            stream.add(ei, game_counter, 0, -1, state, player, env.is_over(), None, obs_ok=ok)
            nsteps = 0
            while not env.is_over():
                legal = legal_ids()
                a = rng.choice(legal) if (env_id == 'no-limit-holdem' or rng.random() < 0.85) else rng.randrange(4)
                act = env._decode_action(a)
                env.timestep += 1
                env.action_recorder.append((env.get_player_id(), act))
                st, player = env.game.step(act)
                state, ok = extract(st)
                done = env.is_over()
                stream.add(ei, game_counter, 1, a, state, player, done, env.get_payoffs() if done else None,
                           obs_ok=ok)
                nsteps += 1
                assert nsteps < 10000
            fin = []
            for p in range(env.num_players):
                f, ok = extract(env.game.get_state(p))
                fin.append((f, ok))
            stream.add_final(game_counter, [f for f, _ in fin], [ok for _, ok in fin])
            game_counter += 1


def gen_nplayer():
    specs = [('leduc-holdem', 'leduc_np', 36, 4, [3, 3, 4, 4, 5, 5], [{}] * 6, 40),
             ('limit-holdem', 'limit_np', 72, 4, [3, 3, 4, 5, 6, 6, 8, 10, 12, 16, 22], [{}] * 11, 30),
             ('no-limit-holdem', 'nolimit_np', 54, 5, [3, 3, 4, 4, 6, 6, 3, 4, 6, 8, 10, 9, 12, 17, 22],
              [{}] * 6 + [{'chips_for_each': 10}, {'chips_for_each': 6, 'dealer_id': 2},
                          {'chips_for_each': 20, 'dealer_id': 5}, {}, {'chips_for_each': 15},
                          {'chips_for_each': 8, 'dealer_id': 7}, {}, {'chips_for_each': 12, 'dealer_id': 16},
                          {'chips_for_each': 30}], 40)]
    for env_id, name, O, A, nps, extra, games in specs:
        seeds = [11 + 17 * i for i in range(len(nps))]
        cfgs = [dict(e, game_num_players=n) for n, e in zip(nps, extra)]
        st = Stream(O, A, max(nps))
        drive_np(env_id, cfgs, seeds, games, st)
        kw = dict(env_np=np.array(nps, dtype=np.int32))
        if env_id == 'no-limit-holdem':
            kw['env_chips'] = np.array([c.get('chips_for_each', 100) for c in cfgs], dtype=np.int32)
            kw['env_dealer'] = np.array([c.get('dealer_id', -1) for c in cfgs], dtype=np.int32)
        st.save(os.path.join(OUT, name + '.npz'), seeds, **kw)
        print('%s.npz: %d events, %d with undefined obs, %d payoff rows' % (
            name, len(st.obs), sum(1 for n in st.ev['obs_len'] if n < 0), sum(st.ev['done'])))


def pick_holdem(rng, state, env):
    legal = sorted(state['legal_actions'].keys())
    if rng.random() < 0.8:
        return rng.choice(legal)
    return rng.randrange(4)          # may be illegal: pins _decode_action (envs/leducholdem.py:81-96)


def gen_leduc():
    seeds = [0, 1, 2, 3, 42, 43, 12941, 2 ** 40 + 9]
    st = Stream(36, 4, 2)
    drive('leduc-holdem', {}, seeds, 60, st, pick_holdem)
    st.save(os.path.join(OUT, 'leduc.npz'), seeds)
    print('leduc.npz: %d events' % len(st.obs))


def gen_limit():
    seeds = [0, 1, 5, 42, 12941, 2 ** 33 + 1]
    st = Stream(72, 4, 2)
    drive('limit-holdem', {}, seeds, 50, st, pick_holdem)
    st.save(os.path.join(OUT, 'limit.npz'), seeds)
    print('limit.npz: %d events' % len(st.obs))


def gen_blackjack():
    seeds = [0, 1, 3, 42, 12941, 777]
    st = Stream(2, 2, 1)

    def pick(rng, state, env):
        return rng.randrange(2)
    drive('blackjack', {}, seeds, 60, st, pick)

    # config 1: examples/run_random.py --env blackjack (env seed 42; set_seed(42) seeds the global np.random that
    # RandomAgent draws from, rlcard/agents/random_agent.py:17-27). set_seed's torch branch is irrelevant here.
    import rlcard
    from rlcard.agents.random_agent import RandomAgent
    env = rlcard.make('blackjack', config={'seed': 42})
    np.random.seed(42)
    agent = RandomAgent(num_actions=env.num_actions)
    env.set_agents([agent for _ in range(env.num_players)])
    traj, payoffs = env.run(is_training=False)
    seq_obs, seq_act = [], []
    for item in traj[0]:
        if isinstance(item, dict):
            seq_obs.append(np.asarray(item['obs'], dtype=np.int64))
            seq_act.append(-1)
        else:
            seq_obs.append(np.zeros(2, dtype=np.int64))
            seq_act.append(int(item))
    st.save(os.path.join(OUT, 'blackjack.npz'), seeds,
            run42_obs=np.stack(seq_obs), run42_act=np.array(seq_act, dtype=np.int32),
            run42_payoffs=np.asarray(payoffs, dtype=np.int64))
    print('blackjack.npz: %d events, run_random(42) trajectory length %d' % (len(st.obs), len(seq_obs)))


def gen_blackjack_shoe():
    """Blackjack beyond one deck / four players (games/blackjack/dealer.py:6-37: deck * num_decks, shuffled, then
    choice(len(deck)) + pop; game.py:15-54 any game_num_players): shoes of 2..8 decks (8 decks = 416 cards, so the
    shuffle and the deals draw random_interval with masks past 8 bits) and tables of 1..7 players, plus the infinite
    deck (0) at 5 players and one deck at 6."""
    cfgs = [(2, 1), (2, 5), (3, 7), (4, 1), (4, 5), (4, 7), (6, 1), (6, 5), (6, 7), (8, 1), (8, 5), (8, 7), (0, 5),
            (1, 6), (5, 3)]
    seeds = [101 + 13 * i for i in range(len(cfgs))]
    configs = [{'game_num_decks': d, 'game_num_players': p} for d, p in cfgs]
    st = Stream(2, 2, max(p for _, p in cfgs))

    def pick(rng, state, env):
        return rng.randrange(2)
    drive('blackjack', configs, seeds, 25, st, pick)
    st.save(os.path.join(OUT, 'blackjack_shoe.npz'), seeds, env_decks=np.array([d for d, _ in cfgs], np.int32),
            env_np=np.array([p for _, p in cfgs], np.int32))
    print('blackjack_shoe.npz: %d events' % len(st.obs))


def gen_doudizhu():
    # 8 seeds x 25 games = 200 games (~12 k events): every seed's stream runs far past its first MT block refills
    seeds = [0, 1, 42, 7, 12941, 2 ** 33 + 1, 99991, 123456789]
    st = Stream(901, 27472, 3, csr_legal=True)

    def pick(rng, state, env):
        return rng.choice(sorted(state['legal_actions'].keys()))
    drive('doudizhu', {}, seeds, 25, st, pick)
    st.save(os.path.join(OUT, 'doudizhu.npz'), seeds)
    print('doudizhu.npz: %d events' % len(st.obs))


def gen_nolimit():
    """No-limit hold'em (rlcard/games/nolimitholdem/, envs/nolimitholdem.py): the default config plus short stacks
    (more all-ins: the bypass deal of game.py:137-171, side-pot judging) and a fixed dealer. Only legal ids are fed:
    the reference's _decode_action fallback names Action.CHECK, which does not exist (envs/nolimitholdem.py:98-100),
    so an illegal id raises there."""
    seeds = [0, 1, 7, 42, 12941, 3, 42, 5, 9]
    cfgs = [{}] * 5 + [{'chips_for_each': 12, 'dealer_id': 1}] * 2 + [{'chips_for_each': 3}, {'chips_for_each': 40,
                                                                                            'dealer_id': 0}]
    st = Stream(54, 5, 2)

    def pick(rng, state, env):
        return rng.choice(sorted(state['legal_actions'].keys()))
    drive('no-limit-holdem', cfgs, seeds, 60, st, pick)
    st.save(os.path.join(OUT, 'nolimit.npz'), seeds,
            env_chips=np.array([c.get('chips_for_each', 100) for c in cfgs], dtype=np.int32),
            env_dealer=np.array([c.get('dealer_id', -1) for c in cfgs], dtype=np.int32))
    print('nolimit.npz: %d events' % len(st.obs))


def gen_cfr():
    """The reference CFRAgent (agents/cfr_agent.py, chance sampling) trained on leduc-holdem envs with
    allow_step_back: its policy / average_policy / regrets dicts (keys = float64 obs bytes, 36 one-hot values) after
    K iterations, as arrays. Deals come from the env's own RandomState (one Env.reset per player per iteration)."""
    import rlcard
    from rlcard.agents.cfr_agent import CFRAgent
    runs = [(0, 25), (5, 12), (42, 40)]
    out = {}
    for r, (seed, iters) in enumerate(runs):
        env = rlcard.make('leduc-holdem', config={'seed': seed, 'allow_step_back': True})
        agent = CFRAgent(env, model_path=os.path.join(WORK, 'cfr_model'))
        for _ in range(iters):
            agent.train()
        for name in ('policy', 'average_policy', 'regrets'):
            d = getattr(agent, name)
            keys = sorted(d.keys())
            obs = np.stack([np.frombuffer(k, dtype=np.float64) for k in keys]).astype(np.uint8)
            assert obs.shape[1] == 36
            out['r%d_%s_obs' % (r, name)] = obs
            out['r%d_%s_val' % (r, name)] = np.stack([np.asarray(d[k], dtype=np.float64) for k in keys])
    np.savez_compressed(os.path.join(OUT, 'cfr.npz'), seeds=np.array([s for s, _ in runs], np.int64),
                        iterations=np.array([k for _, k in runs], np.int64), **out)
    print('cfr.npz: %s' % ', '.join('seed %d x %d it' % x for x in runs))


# --------------------------------------------------------------------------------------------------------------
# The rlcard API's raw side: raw_obs, raw_legal_actions, legal_actions key order, action_record,
# get_perfect_information, get_payoffs (tests/rawcanon.py encodes them as canonical JSON)
# --------------------------------------------------------------------------------------------------------------
class RawStream:
    """Per event: stream index, kind (0 reset, 1 step, 2 step_back, 3 Env.get_state(p) after the game), the action id
    fed (kind 1) or the player asked for (kind 3), the returned player, is_over, and three JSON strings: the state
    view, get_perfect_information() (or the exception it raised) and get_payoffs() (at the step that ends a game;
    called once per game, as Env.run does -- with 3+ hold'em players it may draw from the env's stream)."""

    def __init__(self):
        self.cols = {k: [] for k in ('stream', 'kind', 'act', 'player', 'done')}
        self.state, self.perfect, self.payoffs = [], [], []

    def add(self, si, kind, act, state, player, env, payoffs=None):
        import rawcanon
        if env.name == 'doudizhu':
            from rlcard.games.doudizhu.utils import ACTION_2_ID
            state = rawcanon.ddz_sort_leading(state, ACTION_2_ID)
        for k, v in zip(self.cols, (si, kind, act, player, int(env.is_over()))):
            self.cols[k].append(int(v))
        self.state.append(rawcanon.dumps(rawcanon.state_view(state)))
        try:
            info = env.get_perfect_information()
            if env.name == 'doudizhu':
                info = rawcanon.ddz_sort_perfect(info, ACTION_2_ID)
            self.perfect.append(rawcanon.dumps(info))
        except NotImplementedError:
            self.perfect.append('"NotImplementedError"')
        self.payoffs.append('' if payoffs is None else rawcanon.dumps(payoffs))

    def save(self, path, streams):
        d = {k: np.array(v, dtype=np.int32) for k, v in self.cols.items()}
        d.update(state=np.array(self.state), perfect=np.array(self.perfect), payoffs=np.array(self.payoffs),
                 streams=np.array([json.dumps(s, sort_keys=True) for s in streams]))
        np.savez_compressed(path, **d)


def drive_raw(rec, si, env_id, cfg, seed, games, sb_prob, pick, sb_after_over=0.0):
    """sb_after_over > 0: a finished game is also stepped back with that probability (per check) and play goes on
    from the restored state (Blackjack: Game.step_back puts the last actor's snapshot into the pointer's seat, which
    is seat 0 after the dealer's turn, game.py:125-135)."""
    import random
    import rlcard
    env = rlcard.make(env_id, config=dict(cfg, seed=seed, allow_step_back=sb_prob > 0))
    rng = random.Random(7777 * (si + 1) + seed)
    for _ in range(games):
        state, player = env.reset()
        rec.add(si, 0, -1, state, player, env)
        nsteps = 0
        while True:
            if env.is_over():
                if not (sb_after_over > 0 and rng.random() < sb_after_over):
                    break
                state, player = env.step_back()
                rec.add(si, 2, -1, state, player, env)
                continue
            if sb_prob > 0 and rng.random() < sb_prob:
                r = env.step_back()
                if r is not False:
                    state, player = r
                    rec.add(si, 2, -1, state, player, env)
                    continue
            a = pick(rng, state, env)
            state, player = env.step(a)
            rec.add(si, 1, a, state, player, env, env.get_payoffs() if env.is_over() else None)
            nsteps += 1
            assert nsteps < 10000
        for p in range(env.num_players):
            rec.add(si, 3, p, env.get_state(p), p, env)


def pick_legal(rng, state, env):
    return rng.choice(sorted(state['legal_actions'].keys()))


def gen_raw():
    """raw_<game>.npz: streams (env id config, seed, games, step_back probability) replayed by tests/test_raw.py
    through rlcard_amd.make with the same action ids and step_back calls."""
    specs = {
        'leduc': [('leduc-holdem', {}, 0, 25, 0.0, pick_holdem), ('leduc-holdem', {}, 42, 25, 0.0, pick_holdem),
                  ('leduc-holdem', {}, 3, 12, 0.3, pick_holdem)],
        'limit': [('limit-holdem', {}, 0, 20, 0.0, pick_holdem), ('limit-holdem', {}, 5, 20, 0.0, pick_holdem),
                  ('limit-holdem', {}, 7, 8, 0.3, pick_holdem),
                  ('limit-holdem', {'game_num_players': 4}, 11, 10, 0.0, pick_holdem)],
        'nolimit': [('no-limit-holdem', {}, 0, 20, 0.0, pick_legal),
                    ('no-limit-holdem', {'chips_for_each': 12, 'dealer_id': 1}, 42, 20, 0.0, pick_legal),
                    ('no-limit-holdem', {}, 9, 8, 0.3, pick_legal),
                    ('no-limit-holdem', {'game_num_players': 3, 'chips_for_each': 10}, 13, 12, 0.0, pick_legal),
                    ('no-limit-holdem', {'game_num_players': 6}, 17, 6, 0.0, pick_legal)],
        'blackjack': [('blackjack', {}, 0, 25, 0.0, lambda rng, s, e: rng.randrange(2)),
                      ('blackjack', {}, 42, 25, 0.0, lambda rng, s, e: rng.randrange(2)),
                      ('blackjack', {'game_num_players': 3}, 5, 15, 0.0, lambda rng, s, e: rng.randrange(2)),
                      ('blackjack', {'game_num_players': 5, 'game_num_decks': 6}, 9, 8, 0.0,
                       lambda rng, s, e: rng.randrange(2)),
                      # step_back (game.py:66-70, 125-135): the dealer's RandomState rewinds with its deep copy, the
                      # game's own stream does not (the next game deals from it); the snapshot goes to the current seat
                      ('blackjack', {}, 3, 30, 0.35, lambda rng, s, e: rng.randrange(2), 0.5),
                      ('blackjack', {'game_num_players': 3}, 7, 20, 0.35, lambda rng, s, e: rng.randrange(2), 0.5),
                      ('blackjack', {'game_num_decks': 6}, 11, 20, 0.35, lambda rng, s, e: rng.randrange(2), 0.5),
                      ('blackjack', {'game_num_players': 3, 'game_num_decks': 6}, 13, 15, 0.35,
                       lambda rng, s, e: rng.randrange(2), 0.5)],
        'doudizhu': [('doudizhu', {}, 0, 2, 0.0, pick_legal), ('doudizhu', {}, 42, 1, 0.0, pick_legal),
                     ('doudizhu', {}, 1, 2, 0.25, pick_legal), ('doudizhu', {}, 12941, 2, 0.0, pick_legal)],
    }
    for name, streams in specs.items():
        rec = RawStream()
        meta = []
        for si, (env_id, cfg, seed, games, sb, pick, *after) in enumerate(streams):
            drive_raw(rec, si, env_id, cfg, seed, games, sb, pick, *after)
            meta.append({'env_id': env_id, 'config': cfg, 'seed': seed, 'games': games, 'step_back': sb > 0})
        rec.save(os.path.join(OUT, 'raw_%s.npz' % name), meta)
        print('raw_%s.npz: %d events (%d step_back)' % (name, len(rec.state), rec.cols['kind'].count(2)))


# --------------------------------------------------------------------------------------------------------------
# Hold'em evaluator KATs (compare_hands, rlcard/games/limitholdem/utils.py:526-614)
# --------------------------------------------------------------------------------------------------------------
SUITS = 'SHDC'
RANKS = 'A23456789TJQK'


def card_str(c):           # card index as in limitholdem/card2index.json: suit-major S,H,D,C; rank A..K
    return SUITS[c // 13] + RANKS[c % 13]


def gen_holdem_eval():
    from rlcard.games.limitholdem.utils import compare_hands
    rng = np.random.RandomState(20251015)
    rows, players = [], []
    # (1) random 2-player deals from a full deck
    for _ in range(20000):
        d = rng.permutation(52)[:9]
        rows.append([d[0], d[1], d[4], d[5], d[6], d[7], d[8], d[2], d[3]] + [-1] * 7)
        players.append(2)
    # (2) category-dense deals: restricted decks (few ranks / one suit heavy) and 3 players
    for _ in range(20000):
        nr = rng.randint(4, 9)
        ranks = rng.choice(13, nr, replace=False)
        ns = rng.randint(1, 5)
        suits = rng.choice(4, ns, replace=False)
        deck = np.array([s * 13 + r for s in suits for r in ranks])
        np_ = 3 if rng.rand() < 0.3 else 2
        need = 5 + 2 * np_
        if len(deck) < need:
            extra = np.setdiff1d(np.arange(52), deck)
            deck = np.concatenate([deck, rng.choice(extra, need - len(deck), replace=False)])
        d = rng.permutation(deck)[:need]
        hole = [d[5 + 2 * p: 7 + 2 * p] for p in range(np_)]
        row = list(d[:5])
        for h in hole:
            row += list(h)
        rows.append(row + [-1] * (16 - len(row)))
        players.append(np_)
    # (3) hand-built edge cases: wheel / broadway straights, straight flush vs quads, counterfeited two pair,
    #     three pairs, two trips, flush over straight, split boards
    def c(s):
        return SUITS.index(s[0]) * 13 + RANKS.index(s[1])
    edge = [
        (['SA', 'H2', 'D3', 'C4', 'S9'], [['H5', 'DK'], ['S6', 'C5']]),
        (['ST', 'HJ', 'DQ', 'CK', 'S2'], [['HA', 'D3'], ['C9', 'S8']]),
        (['S5', 'S6', 'S7', 'S8', 'H8'], [['S9', 'D2'], ['D8', 'C8']]),
        (['S2', 'H2', 'D5', 'C5', 'S9'], [['HK', 'DK'], ['CA', 'S3']]),
        (['S2', 'H2', 'D5', 'C5', 'S9'], [['H9', 'DQ'], ['CA', 'D9']]),
        (['S2', 'H2', 'D2', 'C5', 'S5'], [['H5', 'DQ'], ['CA', 'DA']]),
        (['SA', 'SK', 'SQ', 'SJ', 'H4'], [['ST', 'D2'], ['HT', 'DT']]),
        (['S3', 'S7', 'S9', 'H4', 'D5'], [['S6', 'SJ'], ['C6', 'D8']]),
        (['SA', 'HA', 'DA', 'CA', 'SK'], [['HQ', 'DJ'], ['C2', 'D3']]),
        (['S2', 'H3', 'D4', 'C5', 'S6'], [['HK', 'DK'], ['CA', 'SA']]),
        (['SK', 'HK', 'DQ', 'CQ', 'SJ'], [['HJ', 'D2'], ['CA', 'S3']]),
        (['S9', 'H9', 'D9', 'C4', 'S4'], [['H4', 'DA'], ['C9', 'SQ']]),
    ]
    for board, holes in edge:
        row = [c(x) for x in board]
        for h in holes:
            row += [c(x) for x in h]
        rows.append(row + [-1] * (16 - len(row)))
        players.append(len(holes))
    rows = np.array(rows, dtype=np.int8)
    players = np.array(players, dtype=np.int8)
    winners = np.zeros((len(rows), 8), dtype=np.int8)
    for i in range(len(rows)):
        board = [card_str(x) for x in rows[i, :5]]
        hands = []
        for p in range(players[i]):
            hands.append([card_str(x) for x in rows[i, 5 + 2 * p: 7 + 2 * p]] + board)
        w = compare_hands(hands)
        winners[i, :len(w)] = w
    np.savez_compressed(os.path.join(OUT, 'holdem_eval.npz'), cards=rows, players=players, winners=winners)
    print('holdem_eval.npz: %d deals' % len(rows))


def gen_holdem_ref_kats():
    """The reference's own compare_hands known answers (tests/utils/test_holdem_utils.py): its TestHoldemUtils cases
    are run with compare_hands wrapped to record every (hands, winners) pair it asserts on. Hands are 7 card strings
    or None (folded). The tests use a fifth suit letter 'B' and the odd duplicate card; suits only group cards for
    flushes, so each hand's suits are relabelled onto S, H, D, C in order of first appearance, and hands that still
    cannot be 7 distinct cards of a real deck are marked invalid (valid = 0) rather than dropped."""
    import importlib.util
    import unittest
    path = os.path.join(REF, 'tests', 'utils', 'test_holdem_utils.py')
    spec = importlib.util.spec_from_file_location('ref_test_holdem_utils', path)
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    calls = []
    orig = mod.compare_hands

    def rec(hands):
        w = orig(hands)
        calls.append(([None if h is None else list(h) for h in hands], list(w)))
        return w
    mod.compare_hands = rec
    suite = unittest.TestLoader().loadTestsFromTestCase(mod.TestHoldemUtils)
    with open(os.devnull, 'w') as dn:
        res = unittest.TextTestRunner(stream=dn).run(suite)
    m = len(calls)
    maxp = max(len(h) for h, _ in calls)
    cards = np.full((m, maxp, 7), -1, np.int8)
    players = np.zeros(m, np.int8)
    winners = np.zeros((m, maxp), np.int8)
    valid = np.ones(m, np.uint8)
    for i, (hands, w) in enumerate(calls):
        players[i] = len(hands)
        winners[i, :len(w)] = w
        for p, h in enumerate(hands):
            if h is None:
                continue
            order = []
            for c in h:
                if c[0] not in order:
                    order.append(c[0])
            if len(h) != 7 or len(order) > 4:
                valid[i] = 0
                continue
            ids = [SUITS.index('SHDC'[order.index(c[0])]) * 13 + RANKS.index(c[1]) for c in h]
            if len(set(ids)) != 7:
                valid[i] = 0
            cards[i, p] = ids
    np.savez_compressed(os.path.join(OUT, 'holdem_ref_kats.npz'), cards=cards, players=players, winners=winners,
                        valid=valid)
    print('holdem_ref_kats.npz: %d compare_hands calls (%d usable), reference tests run %d, failures %d, errors %d'
          % (m, int(valid.sum()), res.testsRun, len(res.failures), len(res.errors)))


RANK_CHARS = '3456789TJQKA2BR'


def gen_ddz_table():
    """The DouDizhu action-id space (games/doudizhu/jsondata: action_space.txt, card_type.json) as numbers:
    id -> rank counts (3..A,2,B,R), type index, weight. This is the action contract itself (27 472 ids)."""
    from rlcard.games.doudizhu.utils import ID_2_ACTION, ACTION_2_ID, CARD_TYPE, TYPE_CARD
    type_names = list(TYPE_CARD.keys())
    n = len(ID_2_ACTION)
    counts = np.zeros((n, 15), dtype=np.uint8)
    ttype = np.full(n, -1, dtype=np.int16)
    weight = np.full(n, -1, dtype=np.int16)
    for i, a in enumerate(ID_2_ACTION):
        if a == 'pass':
            continue
        for ch in a:
            counts[i, RANK_CHARS.index(ch)] += 1
        (t, w), = CARD_TYPE[0][a]
        ttype[i] = type_names.index(t)
        weight[i] = int(w)
    # position of each id in its type's TYPE_CARD enumeration (weights, then the card lists): the order get_gt_cards
    # (utils.py:225-262) lists a following player's legal actions in; not the id order for trio_solo_chain_2..5
    tc_order = np.zeros(n, dtype=np.int32)
    for t, by_weight in TYPE_CARD.items():
        k = 0
        for _, cards_list in by_weight.items():
            for cards in cards_list:
                tc_order[ACTION_2_ID[cards]] = k
                k += 1
    digest = hashlib.sha256(' '.join(ID_2_ACTION).encode()).hexdigest()
    np.savez_compressed(os.path.join(OUT, 'ddz_actions.npz'), counts=counts, type=ttype, weight=weight, tc_order=tc_order,
                        type_names=np.array(type_names), pass_id=np.int32(ID_2_ACTION.index('pass')),
                        action_space_sha256=np.array(digest))
    print('ddz_actions.npz: %d ids, %d types, sha256 %s' % (n, len(type_names), digest[:16]))


def gen_ddz_judger():
    """Legal sets straight from the reference judger for random hands: leading = playable_cards_from_hand
    (judger.py:124-258), following = get_gt_cards (utils.py:584-621) against a random previous play."""
    from rlcard.games.base import Card
    from rlcard.games.doudizhu.judger import DoudizhuJudger
    from rlcard.games.doudizhu.utils import get_gt_cards, ACTION_2_ID, ID_2_ACTION, cards2str

    class P:                                      # the two attributes get_gt_cards reads
        def __init__(self, hand, played=None):
            self.current_hand, self.played_cards = hand, played

    def hand_of(counts):
        cards = []
        for r, c in enumerate(counts):
            for k in range(c):
                if r == 13:
                    cards.append(Card('BJ', ''))
                elif r == 14:
                    cards.append(Card('RJ', ''))
                else:
                    cards.append(Card('SHDC'[k], RANK_CHARS[r]))
        return cards

    rng = np.random.RandomState(7)
    deck = np.array([r for r in range(13) for _ in range(4)] + [13, 14])
    hands, prev, ptr, ids = [], [], [0], []
    for i in range(3000):
        k = int(rng.choice([1, 2, 3, 4, 5, 8, 12, 17, 20, 20, 20]))
        sel = rng.choice(54, k, replace=False)
        cnt = np.bincount(deck[sel], minlength=15).astype(np.uint8)
        if i % 2 == 0:
            legal = DoudizhuJudger.playable_cards_from_hand(cards2str(hand_of(cnt)))
            p = -1
        else:
            p = int(rng.randint(0, len(ID_2_ACTION) - 1))
            legal = get_gt_cards(P(hand_of(cnt)), P(None, ID_2_ACTION[p]))
        hands.append(cnt)
        prev.append(p)
        ids.extend(sorted(ACTION_2_ID[a] for a in legal))
        ptr.append(len(ids))
    # the reference's own full-deck case (tests/games/test_doudizhu_judger.py:146-156): all 54 cards, leading ->
    # every one of the 27 471 card combos
    full = '3333444455556666777788889999TTTTJJJJQQQQKKKKAAAA2222BR'
    legal = DoudizhuJudger.playable_cards_from_hand(full)
    hands.append(np.array([4] * 13 + [1, 1], np.uint8))
    prev.append(-1)
    ids.extend(sorted(ACTION_2_ID[a] for a in legal))
    ptr.append(len(ids))
    np.savez_compressed(os.path.join(OUT, 'ddz_judger.npz'), hands=np.stack(hands), prev=np.array(prev, np.int32),
                        legal_ptr=np.array(ptr, np.int64), legal_ids=np.array(ids, np.int32))
    print('ddz_judger.npz: %d cases, %d legal ids' % (len(hands), len(ids)))


def pz_record(traj):
    # per agent: [[observation, action_mask, reward, done], action (-1 = None), ...] as JSON lists
    out = {}
    for name, seq in traj.items():
        rec = []
        for k, item in enumerate(seq):
            if k % 2 == 0:
                obs, reward, done = item
                rec.append([np.asarray(obs['observation']).tolist(), np.asarray(obs['action_mask']).tolist(),
                            float(reward), bool(done)])
            else:
                rec.append(-1 if item is None else int(item))
        out[name] = rec
    return out


def gen_pettingzoo():
    # rlcard/utils/pettingzoo_utils.py + agents/pettingzoo_agents.py driven over tests/fake_aec.py (an AEC env of our
    # own; pettingzoo is not installed): episodes (train and eval picks), reorganized transitions, tournament means,
    # wrap_state of AEC observations
    sys.path.insert(0, os.path.dirname(OUT))
    from fake_aec import FakeAEC
    from rlcard.utils.pettingzoo_utils import (wrap_state, run_game_pettingzoo, reorganize_pettingzoo,
                                               tournament_pettingzoo)
    from rlcard.agents.pettingzoo_agents import RandomAgentPettingZoo
    cases = []
    for players, actions, seed in [(2, 4, 1), (3, 5, 2), (4, 3, 7)]:
        env = FakeAEC(players, actions, 4, seed)
        agents = {a: RandomAgentPettingZoo(num_actions=actions) for a in env.possible_agents}
        np.random.seed(seed)
        eps = []
        for e in range(6):
            traj = run_game_pettingzoo(env, agents, is_training=(e % 2 == 0))
            re = reorganize_pettingzoo(traj)
            eps.append({'traj': pz_record(traj),
                        'reorg': {n: [[int(t[1]) if t[1] is not None else -1, float(t[2]), bool(t[4]),
                                       np.asarray(t[0]['observation']).tolist(),
                                       np.asarray(t[3]['observation']).tolist()] for t in ts]
                                  for n, ts in re.items()}})
        tour = tournament_pettingzoo(env, agents, 5)
        cases.append({'players': players, 'actions': actions, 'seed': seed, 'episodes': eps,
                      'tournament': {k: float(v) for k, v in tour.items()}})
    wraps = []
    rng = np.random.RandomState(5)
    for _ in range(8):
        mask = (rng.rand(7) < 0.5).astype(np.int8)
        obs = rng.randint(0, 4, size=3).astype(np.float32)
        w = wrap_state({'observation': obs, 'action_mask': mask})
        wraps.append({'mask': mask.tolist(), 'obs': obs.tolist(), 'legal': [int(x) for x in w['legal_actions']],
                      'raw_legal': [int(x) for x in w['raw_legal_actions']]})
    with open(os.path.join(OUT, 'pettingzoo.json'), 'w') as f:
        json.dump({'cases': cases, 'wrap_state': wraps}, f)
    print('pettingzoo.json', len(cases), 'cases')


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--only', nargs='*', default=None)
    args = ap.parse_args()
    setup_reference()
    gens = {'mt19937': gen_mt, 'leduc': gen_leduc, 'limit': gen_limit, 'blackjack': gen_blackjack,
            'doudizhu': gen_doudizhu, 'nolimit': gen_nolimit, 'cfr': gen_cfr, 'holdem_eval': gen_holdem_eval,
            'holdem_ref_kats': gen_holdem_ref_kats, 'ddz_table': gen_ddz_table,
            'ddz_judger': gen_ddz_judger, 'nplayer': gen_nplayer, 'raw': gen_raw, 'blackjack_shoe': gen_blackjack_shoe,
            'pettingzoo': gen_pettingzoo}
    for name, fn in gens.items():
        if args.only is None or name in args.only:
            fn()


if __name__ == '__main__':
    main()
