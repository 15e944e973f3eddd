"""MultiOptLRs over OptimizeNN: the HIP engine (ce_nn_*) against the oracle.

Two kinds of check, because the observation is a ratio of consecutive
gradients (g_t / |g_{t-1}|, utils_env.py:155-161) and a near-zero gradient
entry turns float32 summation-order noise into an arbitrary ratio:

* state parity with the live oracle (oracle/multinn.py), float32 network
  arithmetic in a different summation order:
    exact      done flags, episode lengths, the composed row order
               (reset + epoch-end shuffles), theta at every reset;
    1e-5       theta and the newest gradient, relative to max |.| of the
               env's vector (north_star's float32 bound); batch loss and
               reward relative;
* observation parity with the live oracle's own rows -- EVERY column: the
  w~, l~ and g~ entries of all H ages (utils_env.py:155-161 over the
  History rings, multioptlrs.py:90-103):
    elementwise  each entry whose denominator is well conditioned (|den| >=
                 1e-3 of its vector's max; at least a quarter qualify) within
                 the engine's MEASURED state differences carried through the
                 ratio, 2 (d_num + |r| d_den) / |den|, plus float32 rounding
                 (clipping to +-100 only shrinks a difference);
    per row      ||d||_inf / ||ref||_inf <= 1e-5 on the agent rows whose
                 every denominator is within 10x of its vector's max and
                 whose ||ref||_inf >= 0.5;
* info parity with the oracle's info dict: batch_loss, weights_mean /
  weights_sum, loss_mean and the terminal loss to 1e-5 relative;
  actions_mean / actions_std (the same float32 learning rates) to 1e-6 /
  1e-4; grads_mean / grads_sum / grad_diff within the measured gradient
  difference; adjusted_loss within its propagated bound;
* formula parity on the engine's own state, as extra checks: every
  observation entry, the loss ratio and the info statistics recomputed in
  numpy from the engine's theta / gradient / loss sequence with the
  reference's formulas (multioptlrs.py:90-127), to float32 rounding of the
  float64 result.
"""
import numpy as np
import pytest

from oracle.multinn import MultiOptLRsNN, nn_draws

pytestmark = pytest.mark.gpu

BOUNDS = 100.0


@pytest.fixture(scope='module', autouse=True)
def _need_gpu():
    import torch
    if not torch.cuda.is_available():
        pytest.fail('GPU tests need a ROCm device (run under gpurun)')


def _iris():
    from custom_envs_amd.data import load_data
    return load_data('iris_synthetic', batch_size=32)


def _ratio(a, b):
    with np.errstate(divide='ignore', invalid='ignore'):
        return np.nan_to_num(np.asarray(a, np.float64) / np.abs(np.asarray(b, np.float64)))


def _obs_form(x):
    return (np.clip(np.nan_to_num(x), -BOUNDS, BOUNDS) - 1).astype(np.float32)


def _run_engine(ds, hidden, seeds, acts, max_batches, H=5):
    from custom_envs_amd.multi_engine import NNMultiEngine
    E = len(seeds)
    eng = NNMultiEngine(E, data_set=ds, hidden=hidden, max_batches=max_batches,
                        max_history=H, seeds=seeds)
    P = eng.n_params
    rec = {'obs0': eng.reset().reshape(E, P, 3 * H), 'state0': eng.get_state(), 'steps': []}
    for t in range(acts.shape[0]):
        out = eng.step(acts[t])
        rec['steps'].append({
            'obs': out['obs'].reshape(E, P, 3 * H).copy(),
            'reward': out['reward'].reshape(E, P).copy(),
            'done': out['done'].reshape(E, P).copy(),
            'info': out['info'].copy(),
            'len': out['episode_len'].copy(),
            'state': eng.get_state()})
    rows = np.asarray(eng.row_agents)
    eng.close()
    return P, rows, rec


def _oracle_rows(obs_o, names):
    if isinstance(obs_o, dict):
        return np.stack([np.asarray(obs_o[n], np.float64) for n in names])
    return np.asarray(obs_o, np.float64)


def _ratio_close(got, want, num, den, d_num, d_den, what):
    """Observation entries clip(num / |den|) - 1 (float32) from the engine vs
    the oracle's own, for one column (one age of w~ or g~, every agent).
    num / den are the ORACLE's vectors; d_num / d_den the max |engine -
    oracle| of the same vectors (measured): an entry's ratio r is then
    within (d_num + |r| d_den) / |den| of the oracle's; twice that plus
    float32 rounding, on the entries with |den| >= 1e-3 max|den| (a quarter
    at least).  Returns the mask of rows with |den| >= 0.1 max|den|."""
    den = np.abs(np.asarray(den, np.float64))
    mask = den >= 1e-3 * den.max()
    assert mask.mean() >= 0.25, (what, mask.mean())
    w = want[mask].astype(np.float64)
    r = np.abs(w + 1)
    tol = 2 * (d_num + r * d_den) / den[mask] + 2.0 ** -22 * (r + 1) + 1e-7
    err = np.abs(got[mask].astype(np.float64) - w)
    assert np.all(err <= tol), (what, float((err - tol).max()), float(err.max()))
    return den >= 0.1 * den.max()


def _check_env(ds, hidden, seed, acts_env, rows, rec, i, max_batches, H=5, state_tol=1e-5,
               stats=None):
    """acts_env: [T][P] actions in row order for env i.  stats (optional
    dict) counts the adjusted_grad comparisons and how many were finite,
    the obs entries compared with the oracle elementwise and the rows
    compared by norm, and the worst row error seen."""
    if stats is None:
        stats = {}
    for key in ('adj_grad', 'adj_grad_finite', 'entries', 'rows', 'row_steps'):
        stats.setdefault(key, 0)
    stats.setdefault('row_err_max', 0.0)
    rows0, slots0 = stats['rows'], stats.get('row_slots', 0)
    P = rows.size
    agent_row = np.empty(P, np.int64)
    agent_row[rows] = np.arange(P)
    env = MultiOptLRsNN(ds.features, ds.targets, hidden=hidden, batch_size=32,
                        max_batches=max_batches, max_history=H)
    env.seed(seed)
    env.reset()
    th0 = nn_draws(seed, env.model.dims, len(ds.features))[0]
    assert np.array_equal(rec['state0']['theta'][i], th0)
    assert np.all(rec['obs0'][i] == -1.0)
    names = env.names

    def snapshot(g_engine, l_engine, th_engine):
        """The oracle's newest raw-history entry and the engine's distance
        from it (max |d| per vector).  A reset entry's loss (and, after an
        auto-reset, its gradient) is not among the engine's outputs: its
        distance is the state bound (state_tol of the vector's max) until the
        first step's loss ratio pins the loss (below)."""
        th_o = np.asarray(env.history['weights'][0], np.float64).copy()
        g_o = np.asarray(env.history['gradients'][0], np.float64).copy()
        l_o = float(np.asarray(env.history['losses'][0], np.float64).reshape(-1)[0])
        d_g = (state_tol * np.abs(g_o).max() + 1e-7 if g_engine is None else
               float(np.abs(np.asarray(g_engine, np.float64) - g_o).max()))
        d_l = state_tol * abs(l_o) if l_engine is None else abs(float(l_engine) - l_o)
        return {'th': th_o, 'g': g_o, 'l': l_o, 'd_g': d_g, 'd_l': d_l,
                'd_th': float(np.abs(np.asarray(th_engine, np.float64) - th_o).max())}

    snaps = [snapshot(rec['state0']['gprev'][i], None, th0)]
    theta_prev = th0.astype(np.float64)
    g_prev = None           # engine gradient of the previous step (None after a reset)
    l_prev = None
    ring = []               # engine's age-0 obs entries of earlier steps this episode
    for t in range(acts_env.shape[0]):
        step = rec['steps'][t]
        act_rows = acts_env[t]
        obs_o, rew_o, done_o, info_o = env.step({names[p]: act_rows[agent_row[p]]
                                                 for p in range(P)})
        # ---- exact: done, episode length, row order
        assert bool(step['done'][i, 0]) == done_o and np.all(step['done'][i] == step['done'][i, 0])
        assert step['len'][i] == info_o['episode']['l']
        st = step['state']
        loss = float(step['info'][i, 1])
        # ---- state parity (float32 network arithmetic, different order)
        th_o = env.model.params
        g_o = env.history['gradients'][0]
        th_e = theta_after = None
        if not done_o:
            th_e = st['theta'][i]
            np.testing.assert_allclose(th_e, th_o, rtol=0,
                                       atol=state_tol * max(np.abs(th_o).max(), 1e-30))
            assert np.array_equal(st['order'][i], env.order()), t
            theta_after = th_e.astype(np.float64)
        g_e = st['gprev'][i]
        np.testing.assert_allclose(g_e, g_o, rtol=0, atol=state_tol * np.abs(g_o).max() + 1e-7)
        assert loss == pytest.approx(float(info_o['batch_loss']), rel=state_tol)
        assert step['reward'][i, 0] == pytest.approx(float(rew_o), rel=state_tol, abs=state_tol)
        # ---- info parity with the oracle's info (multioptlrs.py:112-127)
        info_e = step['info'][i]
        d_g = float(np.abs(np.asarray(g_e, np.float64) - np.asarray(g_o, np.float64)).max())
        assert float(info_e[2]) == pytest.approx(float(info_o['weights_mean']), rel=state_tol)
        assert float(info_e[3]) == pytest.approx(float(info_o['weights_sum']), rel=state_tol)
        assert float(info_e[4]) == pytest.approx(float(info_o['actions_mean']), rel=1e-6)
        assert float(info_e[5]) == pytest.approx(float(info_o['actions_std']), rel=1e-4, abs=1e-9)
        assert float(info_e[10]) == pytest.approx(float(info_o['loss_mean']), rel=state_tol)
        # the ring's 5 gradients are each within the measured difference of
        # the oracle's (the newest is d_g; older ones were checked as newest)
        d_ring = max([d_g] + [sn['d_g'] for sn in snaps[-4:]])
        assert abs(float(info_e[8]) - float(info_o['grads_mean'])) <= 2 * d_ring + 1e-6 * abs(
            float(info_o['grads_mean'])) + 1e-12, t
        assert abs(float(info_e[9]) - float(info_o['grads_sum'])) <= 2 * d_ring * 5 * P + 1e-6 * abs(
            float(info_o['grads_sum'])) + 1e-9, t
        assert abs(float(info_e[13]) - float(info_o['grad_diff'])) <= 2 * (d_g + snaps[-1]['d_g']) + \
            1e-6 * float(info_o['grad_diff']) + 1e-12, t
        if done_o and info_o['loss'] is not None:
            assert float(info_e[0]) == pytest.approx(float(info_o['loss']), rel=state_tol)
        # ---- formula parity on the engine's own sequence
        obs = step['obs'][i][agent_row]            # agent order, [P][3H]
        if done_o:
            # auto-reset: the reset observation, theta back at theta0
            assert np.all(obs == -1.0)
            assert np.array_equal(st['theta'][i], th0)
            env.reset()
            assert np.array_equal(st['order'][i], env.order()), t
            theta_prev, g_prev, l_prev, ring = th0.astype(np.float64), None, None, []
            snaps = [snapshot(None, None, th0)]
            continue
        snaps.append(snapshot(g_e, loss, theta_after))
        if len(snaps) == 2:
            # the reset loss through the engine's first loss ratio
            # (info adjusted_loss = float32(l_1 / |l_0|)): l_0 = l_1 / ratio
            ratio_e = float(step['info'][i, 11])
            if ratio_e != 0 and np.isfinite(ratio_e):
                l0_e = abs(loss / ratio_e)
                snaps[0]['d_l'] = abs(l0_e - abs(snaps[0]['l'])) + 2.0 ** -22 * abs(snaps[0]['l'])
        # ---- observation parity with the oracle's rows: every column, every age
        rows_o = _oracle_rows(obs_o, names)
        stats['row_steps'] += 1
        stats['row_slots'] = stats.get('row_slots', 0) + P
        well = np.ones(P, bool)
        n_age = len(snaps) - 1                   # ages with a ratio this episode
        for k in range(H):
            if k >= n_age:                       # zero-initialised ring: exactly -1
                for col in (k, H + k, 2 * H + k):
                    assert np.all(obs[:, col] == -1.0) and np.all(rows_o[:, col] == -1.0), (t, col)
                continue
            new, old = snaps[-1 - k], snaps[-2 - k]
            well &= _ratio_close(obs[:, k], rows_o[:, k], new['th'], old['th'], new['d_th'],
                                 old['d_th'], ('w', t, k))
            well &= _ratio_close(obs[:, 2 * H + k], rows_o[:, 2 * H + k], new['g'], old['g'],
                                 new['d_g'], old['d_g'], ('g', t, k))
            r = abs(float(rows_o[0, H + k]) + 1)
            tol_l = 2 * (new['d_l'] + r * old['d_l']) / abs(old['l']) + 2.0 ** -22 * (r + 1) + 1e-7
            assert np.all(np.abs(obs[:, H + k].astype(np.float64) - rows_o[:, H + k]) <= tol_l), \
                ('l', t, k)
            stats['entries'] += 2 * P + 1
        ref_inf = np.abs(rows_o).max(axis=1)
        sel = well & (ref_inf >= 0.5)
        if sel.any():
            row_err = np.abs(obs[sel].astype(np.float64) - rows_o[sel]).max(axis=1) / ref_inf[sel]
            stats['rows'] += int(sel.sum())
            stats['row_err_max'] = max(stats['row_err_max'], float(row_err.max()))
            assert row_err.max() <= 1e-5, (t, float(row_err.max()))
        # adjusted_loss (info) against the oracle's, within the l~ bound
        r = abs(float(info_o['adjusted_loss']))
        assert abs(float(info_e[11]) - float(info_o['adjusted_loss'])) <= 2 * (
            snaps[-1]['d_l'] + r * snaps[-2]['d_l']) / abs(snaps[-2]['l']) + 2.0 ** -22 * (r + 1) + 1e-7
        # extra: the engine's own sequence through the reference's formulas
        w_new = _obs_form(_ratio(theta_after, theta_prev))
        assert np.array_equal(obs[:, 0], w_new), t
        if g_prev is not None:
            g_new = _obs_form(_ratio(g_e, g_prev))
            assert np.array_equal(obs[:, 2 * H], g_new), t
            adj_g, dead = _adjusted_grad_mean(g_e, g_prev)
            with np.errstate(over='ignore'):
                finite = np.isfinite(np.float32(adj_g))
            stats['adj_grad'] += 1
            stats['adj_grad_finite'] += int(finite)
            assert finite or dead, t      # a non-finite mean only from a dead-unit ratio
            _close_f32_info(step['info'][i, 12], adj_g, 1e-5)
            _close_f32_info(step['info'][i, 13], np.mean(np.abs(g_e.astype(np.float64) - g_prev)),
                            1e-5, 1e-12)
        if l_prev is not None:
            adj_l = float(_ratio(loss, l_prev))
            _close_f32_info(step['info'][i, 11], adj_l, 1e-6)
            assert np.all(obs[:, H] == _obs_form(adj_l))
        for k, old in enumerate(reversed(ring[-(H - 1):]), start=1):
            assert np.array_equal(obs[:, k], old[:, 0]), (t, k)
            assert np.array_equal(obs[:, 2 * H + k], old[:, 2 * H]), (t, k)
            assert np.all(obs[:, H + k] == old[0, H])
        wsum = np.abs(theta_after).sum()
        assert float(step['info'][i, 3]) == pytest.approx(wsum, rel=1e-6)
        lr = (10.0 ** (act_rows[agent_row].astype(np.float32) - np.float32(4)).astype(np.float64)
              ).astype(np.float32).astype(np.float64)
        assert float(step['info'][i, 4]) == pytest.approx(lr.mean(), rel=1e-6)
        assert float(step['info'][i, 5]) == pytest.approx(lr.std(), rel=1e-4, abs=1e-9)
        ring.append(obs.copy())
        theta_prev, g_prev, l_prev = theta_after, g_e.astype(np.float64), loss
    # the per-row 1e-5 norm bound above is not vacuous for this env: it
    # covered at least 250 (step, row) slots (or a tenth of them on short
    # runs).  The rows that qualify (|den| >= 0.1 max and |ref| >= 0.5) do not
    # grow with the network: measured r06, 489-3090 rows per env over
    # 3,885-407,058 slots (profiles/r06b_nn_row_floor.log)
    n_rows, n_slots = stats['rows'] - rows0, stats.get('row_slots', 0) - slots0
    print('nn env %d per-row check: %d of %d (step, row) slots, worst %.3g'
          % (i, n_rows, n_slots, stats['row_err_max']))
    assert n_rows >= min(250, n_slots // 10), (i, n_rows, n_slots)


def _actions(T, E, P, lo, hi, seed):
    return np.random.RandomState(seed).uniform(lo, hi, (T, E * P)).astype(np.float32)


def _close_f32_info(got, expected, rel, abs_tol=None):
    """Info values are float32 outputs: a float64 mean beyond the float32
    range comes out as +-inf in the reference too, and the engine must
    give the same infinity."""
    with np.errstate(over='ignore'):
        e32 = np.float32(expected)
    if not np.isfinite(e32):
        assert np.float32(got) == e32
    else:
        assert float(got) == pytest.approx(expected, rel=rel, abs=abs_tol)


def _adjusted_grad_mean(g, g_prev):
    """info['adjusted_grad'] = mean |nan_to_num(g / |g_prev|)| (multioptlrs.py:
    115-120, utils_env.py:155-161).  A relu unit that was dead over the
    previous batch has g_prev == 0 exactly for its weights, and where g != 0
    now the ratio is inf -> nan_to_num -> 1.8e308: the reference's own mean
    is then beyond float32 (inf), whatever the other entries are.  Returns
    the mean and whether such an entry explains a non-finite result."""
    g = np.asarray(g, np.float64)
    g_prev = np.asarray(g_prev, np.float64)
    with np.errstate(over='ignore', divide='ignore', invalid='ignore'):
        mean = np.mean(np.abs(_ratio(g, g_prev)))
    return mean, bool(np.any((g_prev == 0) & (g != 0)))


@pytest.mark.parametrize('hidden', [(64,), (96, 32), (32, 64, 128)])
def test_small_networks_against_oracle(hidden):
    """max_batches 7 over 16 steps: two auto-resets, epochs of 5 batches
    (the ragged 22-row batch), split-k forwards (widths < 256)."""
    ds = _iris()
    seeds = [5, 17, 2**33 + 1]
    from custom_envs_amd.multi_engine import NNMultiEngine
    probe = NNMultiEngine(1, data_set=ds, hidden=hidden)
    P = probe.n_params
    probe.close()
    acts = _actions(16, len(seeds), P, 1.0, 2.5, 3)
    P, rows, rec = _run_engine(ds, hidden, seeds, acts, max_batches=7)
    for i, seed in enumerate(seeds):
        _check_env(ds, hidden, seed, acts[:, i * P:(i + 1) * P], rows, rec, i, 7)


def test_long_run_small_network_against_oracle():
    """64 steps with max_batches 11: five auto-resets and a dozen epoch ends
    (each a reshuffle composed into the row order), the rings wrapping many
    times, three envs against live oracle envs."""
    ds = _iris()
    seeds = [2, 31, 77]
    hidden = (32,)
    P = 4 * 32 + 32 + 32 * 3 + 3
    acts = _actions(64, len(seeds), P, 1.0, 2.5, 12)
    _, rows, rec = _run_engine(ds, hidden, seeds, acts, max_batches=11)
    for i, seed in enumerate(seeds):
        _check_env(ds, hidden, seed, acts[:, i * P:(i + 1) * P], rows, rec, i, 11)


def test_many_classes_against_oracle():
    """7 classes (past the eval kernels' compiled 4-class instance, nn_km):
    the 32-class-bound instance of nn_grad_kernel / nn_step_kernel, with a
    hidden width (96) that does not divide the 512-thread block."""
    from custom_envs_amd.data import normalize, to_onehot
    from custom_envs_amd.dataset import InMemoryDataSet
    rs = np.random.RandomState(3)
    labels = np.repeat(np.arange(7), 20)
    feats = rs.normal(labels[:, None] * 0.5, 1.0, (140, 5))
    ds = InMemoryDataSet(normalize(feats), to_onehot(labels)[0], 32)
    seeds = [6, 11]
    hidden = (96, 64)
    P = 5 * 96 + 96 + 96 * 64 + 64 + 64 * 7 + 7
    acts = _actions(12, len(seeds), P, 1.0, 2.5, 8)
    P2, rows, rec = _run_engine(ds, hidden, seeds, acts, max_batches=9)
    assert P2 == P
    for i, seed in enumerate(seeds):
        _check_env(ds, hidden, seed, acts[:, i * P:(i + 1) * P], rows, rec, i, 9)


def test_long_history_against_oracle():
    """max_history 10: ring ages past the 8 the agent kernel keeps in
    registers are loaded at staging time."""
    ds = _iris()
    seeds = [4, 8]
    hidden = (32,)
    P = 4 * 32 + 32 + 32 * 3 + 3
    acts = _actions(16, len(seeds), P, 1.0, 2.5, 6)
    _, rows, rec = _run_engine(ds, hidden, seeds, acts, max_batches=13, H=10)
    for i, seed in enumerate(seeds):
        _check_env(ds, hidden, seed, acts[:, i * P:(i + 1) * P], rows, rec, i, 13, H=10)


def test_default_network_against_oracle():
    """get_problem('nn') defaults: create_neural_net (256, 256) over the
    iris-shaped set, P = 67,843 agents per env."""
    ds = _iris()
    seeds = [0, 9]
    hidden = (256, 256)
    P = 4 * 256 + 256 + 256 * 256 + 256 + 256 * 3 + 3
    acts = _actions(6, len(seeds), P, 1.0, 2.5, 4)
    P2, rows, rec = _run_engine(ds, hidden, seeds, acts, max_batches=400)
    assert P2 == P
    for i, seed in enumerate(seeds):
        _check_env(ds, hidden, seed, acts[:, i * P:(i + 1) * P], rows, rec, i, 400)


def test_default_network_benchmark_size_sampled_envs():
    """The NN bench line's size: 1024 envs of the default (256, 256) network
    (P = 67,843 agents each, device-resident actions and outputs as in
    bench.py); envs 0 and 1023 of the grid against live oracle envs over 12
    steps, which cross two epoch ends of the 150-row set (ragged 22-row
    batch, reshuffle)."""
    import torch
    from custom_envs_amd.multi_engine import NNMultiEngine
    ds = _iris()
    E, H, T = 1024, 5, 12
    hidden = (256, 256)
    sample = [0, 1023]
    eng = NNMultiEngine(E, data_set=ds, hidden=hidden, max_batches=400, max_history=H,
                        seeds=list(range(E)))
    P = eng.n_params
    assert P == 4 * 256 + 256 + 256 * 256 + 256 + 256 * 3 + 3
    rows = np.asarray(eng.row_agents)
    out = eng.alloc_device_outputs()
    eng.reset_device(out)
    eng.wait()

    def pick(st):
        return {k: (v[sample] if getattr(v, 'ndim', 0) and v.shape[0] == E else v)
                for k, v in st.items()}

    obs0 = out['obs'].view(E, P, 3 * H)[sample].cpu().numpy()
    rec = {'obs0': obs0, 'state0': pick(eng.get_state()), 'steps': []}
    gen = torch.Generator(device='cuda')
    gen.manual_seed(99)
    acts = torch.empty(E * P, dtype=torch.float32, device='cuda')
    acts_s = np.zeros((T, len(sample), P), np.float32)
    for t in range(T):
        acts.uniform_(1.0, 2.5, generator=gen)
        torch.cuda.synchronize()
        eng.step_device(acts, out)
        eng.wait()
        av = acts.view(E, P)
        for k, e in enumerate(sample):
            acts_s[t, k] = av[e].cpu().numpy()
        rec['steps'].append({
            'obs': out['obs'].view(E, P, 3 * H)[sample].cpu().numpy(),
            'reward': out['reward'].view(E, P)[sample].cpu().numpy(),
            'done': out['done'].view(E, P)[sample].cpu().numpy(),
            'info': out['info'].view(E, -1)[sample].cpu().numpy(),
            'len': out['episode_len'][sample].cpu().numpy(),
            'state': pick(eng.get_state())})
    eng.close()
    stats = {}
    for k, e in enumerate(sample):
        _check_env(ds, hidden, e, acts_s[:, k], rows, rec, k, 400, stats=stats)
    print('nn per-row check:', {k: stats[k] for k in ('rows', 'row_steps', 'row_slots', 'row_err_max')})
    assert stats['adj_grad'] >= 2 * (T - 2)
    # the per-row 1e-5 norm bound is not vacuous: 250 rows per sampled env
    assert stats['row_steps'] >= 2 * (T - 2)
    assert stats['rows'] >= 250 * len(sample), stats


def test_divergence_stops_early_with_penalty():
    """multioptlrs.py:105-107: loss > 1e4 ends the episode with reward
    reduced by (max_batches - step); lr 1e2..1e4 drives the loss there."""
    ds = _iris()
    from custom_envs_amd.multi_engine import NNMultiEngine
    hidden = (64,)
    eng = NNMultiEngine(2, data_set=ds, hidden=hidden, max_batches=50, seeds=[1, 2])
    P = eng.n_params
    eng.reset()
    acts = _actions(12, 2, P, 6.0, 8.0, 5)
    oracles = []
    for seed in (1, 2):
        env = MultiOptLRsNN(ds.features, ds.targets, hidden=hidden, max_batches=50)
        env.seed(seed)
        env.reset()
        oracles.append(env)
    rows = np.asarray(eng.row_agents)
    agent_row = np.empty(P, np.int64)
    agent_row[rows] = np.arange(P)
    early = 0
    for t in range(12):
        out = eng.step(acts[t])
        for i, env in enumerate(oracles):
            a = acts[t, i * P:(i + 1) * P]
            _, rew, done, info = env.step({env.names[p]: a[agent_row[p]] for p in range(P)})
            assert bool(out['done'][i * P]) == done
            assert out['episode_len'][i] == info['episode']['l']
            if done:
                early += info['episode']['l'] < 50
                if np.isfinite(rew):
                    assert out['reward'][i * P] == pytest.approx(float(rew), rel=1e-3, abs=1e-3)
                env.reset()
    eng.close()
    assert early > 0


def test_optvecenv_and_single_env_surface():
    """OptVecEnv over make('MultiOptLRs-v0', problem='nn', ...) runs on one
    engine; rows are env-major in sorted agent-name order; the single env
    returns the reference's Dict surface."""
    import functools
    import custom_envs_amd
    from custom_envs_amd.vectorize.optvecenv import OptVecEnv
    ds = _iris()
    fn = functools.partial(custom_envs_amd.make, 'MultiOptLRs-v0', problem='nn',
                           data_set=ds, hidden=(32,), max_batches=5)
    venv = OptVecEnv([fn] * 3)
    assert venv.engine_backed
    P = 4 * 32 + 32 + 32 * 3 + 3
    assert venv.num_envs == 3 * P and venv.agent_no_list == [P] * 3
    obs = venv.reset()
    assert obs.shape == (3 * P, 15) and np.all(obs == -1)
    for t in range(6):
        states, rewards, terminals, infos = venv.step(np.full(3 * P, 1.5, np.float32))
        assert states.shape == (3 * P, 15) and len(infos) == 3 * P
        assert np.all(terminals == (t == 4))
    venv.close()
    env = custom_envs_amd.make('MultiOptLRs-v0', problem='nn', data_set=ds, hidden=(32,))
    env.seed(3)
    state = env.reset()
    assert len(state) == P and all(np.all(v == -1) for v in state.values())
    state, reward, terminal, info = env.step({n: np.float32(1.5) for n in state})
    assert isinstance(reward, float) and isinstance(terminal, bool)
    assert info['loss'] is None and set(info) >= {'batch_loss', 'grads_mean', 'episode'}
    env.close()


def test_device_path_and_graphs_match_host_path():
    """step_device / step_many_device (hipGraph of k steps) give the host
    path's outputs bit for bit; graphs of odd k start at alternating
    ping-pong parities (captured per parity)."""
    import torch
    from custom_envs_amd.multi_engine import NNMultiEngine
    ds = _iris()
    kw = dict(data_set=ds, hidden=(64,), max_batches=5, seeds=[7, 8, 9])
    host = NNMultiEngine(3, **kw)
    dev = NNMultiEngine(3, **kw)
    P = host.n_params
    T = 11
    acts = _actions(T, 3, P, 1.0, 2.5, 9)
    host.reset()
    ref = []
    for t in range(T):
        o = host.step(acts[t])
        ref.append({k: v.copy() for k, v in o.items()})
    stream = torch.cuda.Stream()
    torch.cuda.set_stream(stream)
    dev.set_stream(stream.cuda_stream)
    out = dev.alloc_device_outputs()
    dev.reset_device(out)
    dacts = torch.from_numpy(acts).cuda()
    t = 0
    for k in (1, 3, 3, 1, 3):          # parities 0, 1, 0, 1, 0 at graph starts
        if k == 1:
            dev.step_device(dacts[t], out)
        else:
            dev.step_many_device(k, dacts[t:], out)
        torch.cuda.synchronize()
        t += k
        got = {n: v.cpu().numpy() for n, v in out.items()}
        r = ref[t - 1]
        assert np.array_equal(got['obs'].reshape(r['obs'].shape), r['obs']), t
        assert np.array_equal(got['reward'], r['reward'])
        assert np.array_equal(got['done'], r['done'])
        assert np.array_equal(got['episode_len'], r['episode_len'])
        np.testing.assert_array_equal(got['info'], r['info'])
    assert np.array_equal(host.get_state()['theta'], dev.get_state()['theta'])
    host.close()
    dev.close()

