"""Parity past the MT19937 refills, at the shapes bench.py times.

A freshly seeded lane-game env (Leduc, Limit, No-limit, Blackjack) holds ring blocks 0..SLOTS-2 and first refills once
its stream is inside block L (position >= rng_period - 2 x 624: 3 744 draws with 8 slots, cs_ring.h `needs_refill`),
then every (SLOTS - 1) x 624 draws; DouDizhu's two-block word
window first twists at ~1 184 draws (cs_doudizhu.hip `WaveMt::window`). The tests below drive every env well past
two refills and compare every launch with the CPU oracle, so the paths the timed launches run in steady state
(ring_refill_wave's multi-block twist, ring_gen_serial, the batched restage after a refill, Leduc's reset_swar across block
edges, DouDizhu's mt_twist_wave and the MT_WORDS wrap) are all checked bit-exactly.
Reference: the deals that consume the stream, rlcard/games/leducholdem/game.py:46-95, doudizhu/dealer.py:12-76,
limitholdem/dealer.py:11-21; numpy RandomState (MT19937 legacy)."""
import numpy as np
import pytest

from rlcard_amd import seeding
from test_gpu_engine import _assert_same, _np, _oracle_batch, _vec

torch = pytest.importorskip('torch')
pytestmark = pytest.mark.gpu



def past_refills(k):
    """min draws per env: past the first refill and k more (from the library's ring geometry)"""
    return lambda v: v.rng_first_refill + k * (v.rng_period - 624)


@pytest.fixture(scope='module', autouse=True)
def _need_gpu():
    if not torch.cuda.is_available():
        pytest.fail('GPU tests need a visible GPU (run them on the MI355X box)')


def _draws(ob, n):
    return np.array([ob.draws(i) for i in range(n)], np.int64)


def _roll_past_refills(oracle, game, n, T, launches, flags, seed, min_draws):
    v = _vec(game, n, seed=seed)
    v.set_kernel_flags(flags)
    ob = _oracle_batch(oracle, game, range(seed, seed + n))
    _assert_same(_np(v.reset()), ob.reset(), 'reset')
    out = v.new_traj_out(T)           # one buffer reused across launches, as bench.py does
    for c in range(launches):
        got = _np(v.rollout(T, policy_seed=5, t0=c * T, out=out))
        exp = ob.rollout(T, 5, c * T, 0)
        _assert_same(got, exp, '%s flags %d launch %d' % (game, flags, c))
    torch.cuda.synchronize()
    d = _draws(ob, n)
    min_draws = min_draws(v) if callable(min_draws) else min_draws
    assert d.min() >= min_draws, 'test too short: min draws %d < %d' % (d.min(), min_draws)
    for i in sorted({0, 1, 63, 64, n // 2, n - 1, int(np.argmax(d)), int(np.argmin(d))} & set(range(n))):
        assert v.rng_position(i) == d[i] % v.rng_period, i
    return v, ob


@pytest.mark.parametrize('flags', [0, 1])          # 1 = serial (per-lane) refill instead of the wave twist
def test_leduc_bench_shape_past_refills(oracle, flags):
    """bench.py's Leduc sequence (T = 256 fused steps, one trajectory buffer) on 4 133 envs (a ragged tail wave)
    for 28 launches: every env crosses the first refill and one full refill cycle after it (>= 18 096 draws)."""
    _roll_past_refills(oracle, 'leduc-holdem', 4096 + 37, 256, 28, flags, 42, past_refills(1))


@pytest.mark.parametrize('game,T,launches', [('limit-holdem', 128, 10), ('no-limit-holdem', 128, 10),
                                             ('blackjack', 64, 9)])
def test_lane_games_bench_shape_past_refills(oracle, game, T, launches):
    """The other lane-per-env games at their bench T: each env draws ~25-57 words per step, so a few launches
    cross several refills (every slot of the ring is rewritten at least twice)."""
    _roll_past_refills(oracle, game, 2048 + 19, T, launches, 0, 42, past_refills(2))


def test_doudizhu_past_mt_twists(oracle):
    """64 DouDizhu envs for 22 x 64 = 1 408 steps: every env crosses its first mt_twist_wave (~1 184 draws) and the
    MT_WORDS position wrap (>= 1 426 draws each)."""
    _roll_past_refills(oracle, 'doudizhu', 64, 64, 22, 0, 42, 1300)


def test_leduc_full_size_after_precondition(oracle):
    """The bench's 2^20 Leduc envs after 14 preconditioning launches (T = 256): one timed-shape launch is then
    compared with the oracle on three windows (start, middle, end) replayed from seeding with the same env ids."""
    n, T, win, pre = 1 << 20, 256, 256, 14
    v = _vec('leduc-holdem', n, seed=42)
    v.reset()
    out = v.new_traj_out(T)
    for c in range(pre):
        v.rollout(T, policy_seed=5, t0=c * T, out=out)
    tr = v.rollout(T, policy_seed=5, t0=pre * T, out=out)
    torch.cuda.synchronize()
    for start in (0, n // 2 + 17, n - win):
        ob = _oracle_batch(oracle, 'leduc-holdem', range(42 + start, 42 + start + win))
        ob.reset()
        for c in range(pre):
            ob.rollout(T, 5, c * T, start)
        exp = ob.rollout(T, 5, pre * T, start)
        got = {k: x[:, start:start + win].cpu().numpy() for k, x in tr.items()}
        _assert_same(got, exp, 'window %d' % start)
        d = _draws(ob, win)
        assert d.min() >= v.rng_first_refill + 300, 'window %d has not refilled (min draws %d)' % (start, d.min())
        for i in (0, win - 1):
            assert v.rng_position(start + i) == d[i] % v.rng_period


def test_cfr_batched_past_refills(oracle):
    """Batched chance-sampling CFR for enough iterations that every env's stream refills (each iteration deals once
    per player): tables to 1e-9, RNG positions exactly."""
    from rlcard_amd import VecEnv
    from rlcard_amd.agents import CFRAgent
    B, K = 256 + 3, 400
    v = VecEnv('leduc-holdem', B, seed=21)
    agent = CFRAgent(v)
    agent.train(K)
    torch.cuda.synchronize()
    keys, lens = seeding.seed_keys(range(21, 21 + B))
    c = oracle.CFR(keys, lens)
    c.train(K)
    d = np.array([c.draws(i) for i in range(B)])
    # env e's first refill comes after (e % 15) x 624 draws (cs_ring.h seed_blocks): most streams are past it
    first = (np.arange(B) % 15) * 624
    assert (d >= first + 300).mean() > 0.5, (d - first).min()
    t = c.tables()
    host = agent._tables()
    assert np.array_equal(host['flags'].astype(np.uint8), t['flags'])
    for name, bit in (('policy', 1), ('average_policy', 2), ('regrets', 2)):
        rows = (t['flags'] & bit) != 0
        # fp64 atomics add the 259 deals of an iteration in any order, so the rounding differences grow with the
        # iterations: 1e-9 holds at K = 400 (at 700-800, 1e-8 absolute on a policy entry near zero was seen)
        np.testing.assert_allclose(host[name][rows], t[name][rows], rtol=1e-9, atol=1e-9 * np.abs(t[name]).max(),
                                   err_msg=name)
    for i in (0, 1, 63, 64, B // 2, B - 1):
        assert v.rng_position(i) == d[i] % v.rng_period
