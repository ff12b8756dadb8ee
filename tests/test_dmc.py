"""DMC on the device (rlcard_amd/agents/dmc_agent.py, rlcard_amd/csrc/cs_dmc.hip) vs restatements of the reference:
the actor-buffer loop of rlcard/agents/dmc_agent/utils.py:97-163 (act) and get_batch (:33-46), and DMCNet.forward
(model.py:21-43) in plain torch fp32. Needs a GPU."""
import numpy as np
import pytest

torch = pytest.importorskip('torch')
pytestmark = pytest.mark.gpu


@pytest.fixture(scope='module', autouse=True)
def _need_gpu():
    if not torch.cuda.is_available():
        pytest.fail('GPU tests need a visible GPU (run them on the MI355X box)')


def ref_act(traj, P, T, feature):
    """utils.py:97-163 restated over rollout rows: per env, per player, the streams act builds and the chunks it
    emits (`while size[p] > T`), in emission order. traj: numpy dict of [L][n] rows."""
    L, n = traj['player'].shape
    chunks = {}
    for e in range(n):
        buf = {p: dict(done=[], episode_return=[], target=[], state=[], action=[]) for p in range(P)}
        rows = {p: [] for p in range(P)}
        for t in range(L):
            p = int(traj['player'][t, e])
            if p < P:
                rows[p].append(t)
            if traj['done'][t, e]:
                for q in range(P):
                    r, diff = rows[q], len(rows[q])
                    if diff > 0:
                        pay = float(traj['reward'][t, e, q])
                        b = buf[q]
                        b['done'] += [False] * (diff - 1) + [True]
                        b['episode_return'] += [0.0] * (diff - 1) + [pay]
                        b['target'] += [pay] * diff
                        b['state'] += [traj['obs'][x, e] for x in r]
                        b['action'] += [feature(int(traj['action'][x, e])) for x in r]
                    rows[q] = []
                    while len(buf[q]['target']) > T:
                        chunks.setdefault((e, q), []).append({k: v[:T] for k, v in buf[q].items()})
                        for k in buf[q]:
                            buf[q][k] = buf[q][k][T:]
    return chunks


@pytest.mark.parametrize('game,n,T_roll,launches,Tc', [('leduc-holdem', 300, 64, 6, 20), ('blackjack', 200, 32, 5, 10),
                                                       ('doudizhu', 40, 32, 8, 25), ('limit-holdem', 150, 48, 5, 30),
                                                       ('no-limit-holdem', 100, 40, 4, 16)])
def test_actor_buffers_match_reference_act_loop(game, n, T_roll, launches, Tc):
    from rlcard_amd import VecEnv
    from rlcard_amd.agents.dmc_agent import ActorBuffers, shapes_of
    v = VecEnv(game, n, seed=11)
    v.reset()
    buf = ActorBuffers(v, T=Tc, slots=3 + (T_roll + Tc - 1) // Tc)
    P = v.num_players
    feats = v.action_features(torch.arange(v.num_actions, device=v.device)).cpu().numpy().astype(np.int8)
    state_shape, _ = shapes_of(v)
    got = {}
    rows = []
    for c in range(launches):
        tr = v.rollout(T_roll, policy_seed=4, t0=c * T_roll)
        rows.append({k: x.cpu().numpy() for k, x in tr.items()})
        ready = buf.fill(tr)
        ready_np = ready.cpu().numpy()
        assert np.all(np.diff(ready_np // buf.slots) >= 0), 'ready chunks in (env, player) order'
        pl = buf.player_of(ready)
        for p in range(P):
            ids = ready[pl == p]
            b = {k: x.cpu().numpy() for k, x in buf.get_batch(p, ids).items()}
            for j, cid in enumerate(ids.cpu().numpy()):
                e = int(cid // buf.slots) // P
                got.setdefault((e, p), []).append({k: b[k][:, j] for k in b})
    assert not buf.dropped()
    traj = {k: np.concatenate([r[k] for r in rows], axis=0) for k in rows[0]}
    exp = ref_act(traj, P, Tc, lambda a: feats[a])
    assert set(got) == set(exp) and len(exp) > 0
    for key, chunks in exp.items():
        assert len(got[key]) == len(chunks), key
        for g, x in zip(got[key], chunks):
            sd = state_shape[key[1]][0]
            assert np.array_equal(g['state'], np.stack(x['state'])[:, :sd].astype(np.int8)), key
            assert np.array_equal(g['action'], np.stack(x['action'])), key
            assert np.array_equal(g['target'], np.array(x['target'], np.float32)), key
            assert np.array_equal(g['episode_return'], np.array(x['episode_return'], np.float32)), key
            assert np.array_equal(g['done'], np.array(x['done'])), key


@pytest.mark.parametrize('game', ['leduc-holdem', 'doudizhu', 'no-limit-holdem'])
def test_q_values_match_dmcnet_forward(game):
    """Fused first layer + GEMMs == DMCNet.forward on [obs, action feature] (fp32; tolerance for the different
    summation order of the split first layer); greedy selection == argmax per state."""
    from rlcard_amd import VecEnv
    from rlcard_amd.agents.dmc_agent import DMCNet, q_values, select_actions, shapes_of
    torch.manual_seed(0)
    n = 64 if game == 'doudizhu' else 512
    v = VecEnv(game, n, seed=3)
    v.reset()
    tr = v.rollout(8, policy_seed=1)
    st = {k: tr[k][-1] for k in ('obs', 'legal', 'player')}
    counts, offsets, ids = v.legal_lists(st['legal'])
    state_of = torch.repeat_interleave(torch.arange(n, device=ids.device, dtype=torch.int32), counts.long())
    state_shape, action_shape = shapes_of(v)
    p = 1 if game == 'doudizhu' else 0
    net = DMCNet(state_shape[p], action_shape[p]).cuda()
    got = q_values(v, net, st['obs'], state_of, ids)
    feats = v.action_features(ids).float()
    with torch.no_grad():
        exp = net(st['obs'][state_of.long(), :state_shape[p][0]].float(), feats)
    torch.testing.assert_close(got, exp, rtol=1e-5, atol=1e-5)
    acts = select_actions(got, counts, offsets, ids).cpu().numpy()
    g, o, c, i = got.cpu().numpy(), offsets.cpu().numpy(), counts.cpu().numpy(), ids.cpu().numpy()
    for s in range(n):
        seg = g[o[s]:o[s] + c[s]]
        assert acts[s] == i[o[s] + int(np.argmax(seg))]
    # epsilon 1: uniform legal ids
    acts = select_actions(got, counts, offsets, ids, eps=1.0, seed=9, t=3).cpu().numpy()
    for s in range(n):
        assert acts[s] in set(i[o[s]:o[s] + c[s]].tolist())


def test_dmc_actor_fills_learner_batches():
    """The vectorised act loop on DouDizhu: device policy, lazy resets marked as non-transitions, chunks handed out
    as [T, B, ...] batches of the reference's shapes and dtypes."""
    from rlcard_amd import VecEnv
    from rlcard_amd.agents.dmc_agent import DMCActor, DMCModel, shapes_of
    v = VecEnv('doudizhu', 32, seed=5)
    ss, acs = shapes_of(v)
    model = DMCModel(ss, acs, mlp_layers=(64, 64), exp_epsilon=0.1)
    actor = DMCActor(v, model, T=20, steps_per_fill=40)
    total = {p: 0 for p in range(3)}
    for _ in range(4):
        ready = actor.act()
        for p, ids in ready.items():
            b = actor.buffers.get_batch(p, ids)
            assert b['state'].shape == (20, ids.numel(), ss[p][0]) and b['state'].dtype == torch.int8
            assert b['action'].shape == (20, ids.numel(), 54)
            if ids.numel():
                assert bool(torch.isfinite(b['target']).all())
                assert bool(((b['target'] == 0) | (b['target'] == 1)).all())
            total[p] += ids.numel()
    assert not actor.buffers.dropped()
    assert sum(total.values()) > 0


def test_actor_buffers_overflow_raises_and_lists_no_stale_chunk():
    """A ring too small for one fill (slots = 2, chunks never gathered): rows that would overwrite a chunk not yet
    handed out are dropped, not counted (no listed chunk holds one) and fill() raises."""
    from rlcard_amd import VecEnv, _abi
    from rlcard_amd.agents.dmc_agent import ActorBuffers
    v = VecEnv('leduc-holdem', 64, seed=5)
    v.reset()
    buf = ActorBuffers(v, T=4, slots=2)
    tr = v.rollout(6, policy_seed=1)
    ready = buf.fill(tr)                     # <= 6 rows per (env, player): fits the two 4-row chunks
    assert not buf.dropped()
    assert int(ready.numel()) <= 64 * 2 * 2
    with pytest.raises(_abi.CardsimError, match='overflowed'):
        for k in range(4):
            buf.fill(v.rollout(64, policy_seed=1, t0=6 + 64 * k))
    assert buf.dropped()
