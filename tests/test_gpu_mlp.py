"""Optimize-v0 over the config-3 MLP: HIP engine vs the oracle.

Tolerances (north star: "within 1e-5 relative for fp32 observations/
rewards"): the model is float32 on both sides, but the engine sums on MFMA
(k-ordered fma chains, partial sums per wave) while numpy calls BLAS sgemm,
so values agree to float32 rounding of differently ordered sums:
  - exact: done, episode length, W0 (native MT19937 vs numpy), the float32
    weights after W <- W - a (the update is one f32 subtraction on both
    sides), the zero weight-history block of obs;
  - obs row: ||d||_inf <= 1e-5 ||ref||_inf (gradient entries near zero come
    out of cancelling sums over 32 samples);
  - reward = -loss, objective and L' = obs[P]: 1e-5 relative;
  - accuracy: the count of correct argmax rows may differ only where two
    logits tie to float32 rounding; asserted exact on these problems.
"""
import numpy as np
import pytest

from conftest import golden
from oracle.optimize import Optimize as OracleEnv

pytestmark = pytest.mark.gpu

RTOL = 1e-5


@pytest.fixture(scope='module', autouse=True)
def _need_gpu():
    import torch
    if not torch.cuda.is_available():
        pytest.fail('GPU tests need a ROCm device (run under gpurun)')


def _engine(features, targets, num_envs, auto_reset=True):
    from custom_envs_amd.engine import OptimizeEngine
    return OptimizeEngine(features, targets, num_envs=num_envs, batch_size=32, model='mlp',
                          auto_reset=auto_reset)


def _row_close(got, ref, tol=RTOL, what=''):
    got = np.asarray(got, np.float64)
    ref = np.asarray(ref, np.float64)
    scale = max(np.abs(ref).max(), 1e-30)
    diff = np.abs(got - ref)
    err = diff.max() / scale
    i = int(diff.argmax())
    assert err <= tol, '%s err %.3g at %d of %d: got %r ref %r (row max %.4g at %d)' % (
        what, err, i, len(ref), got[i], ref[i], scale, int(np.abs(ref).argmax()))


def _rel(got, ref):
    return abs(float(got) - float(ref)) / max(abs(float(ref)), 1e-30)


@pytest.mark.parametrize('seed', [5, 6])
def test_golden_mlp_rollout(seed):
    from oracle.gen_golden import mlp_actions
    data = golden('mlp_data_128x16.npz')
    fx = golden('optimize_mlp_s%d.npz' % seed)
    eng = _engine(data['features'], data['targets'], 1)
    try:
        P = eng.act_dim
        assert P == 16 * 64 + 64 + 64 * 10 + 10
        eng.seed([seed])
        reset = eng.reset()
        assert np.array_equal(reset[0], fx['reset_obs'])
        assert np.array_equal(eng.get_state()['init_weights'][0].astype(np.float32),
                              fx['init_weights'])
        acts = mlp_actions(int(fx['action_seed']), len(fx['reward']), P)
        keep = list(fx['keep'])
        for t in range(len(fx['reward'])):
            out = eng.step(acts[t:t + 1])
            assert bool(out['done'][0]) == bool(fx['done'][t]), t
            assert int(out['episode_len'][0]) == int(fx['ep_len'][t]), t
            assert _rel(out['reward'][0], fx['reward'][t]) <= RTOL, t
            assert _rel(out['objective'][0], fx['objective'][t]) <= RTOL, t
            assert out['accuracy'][0] == np.float32(fx['accuracy'][t]), t
            assert _rel(out['obs'][0][P], fx['loss_obs'][t]) <= RTOL, t
            if t in keep:
                k = keep.index(t)
                _row_close(out['obs'][0], fx['obs'][k])
                if not fx['done'][t]:
                    assert not out['obs'][0][:P].any()
                    w = eng.get_state()['weights'][0].astype(np.float32)
                    assert np.array_equal(w, fx['weights'][k]), t
    finally:
        eng.close()


def test_config3_envs_against_live_oracle():
    """Full config-3 shapes (784 -> 64 -> 10, N = 1024, B = 32), 3 envs across
    an auto-reset, each against its own oracle env."""
    from custom_envs_amd.data import load_data
    seq = load_data('mnist_synthetic', batch_size=32)
    seeds = [0, 1, 2]
    eng = _engine(seq.features, seq.targets, len(seeds))
    refs = []
    for s in seeds:
        env = OracleEnv(seq.features, seq.targets, batch_size=32, model='mlp')
        env.seed(s)
        env.reset()
        refs.append(env)
    try:
        eng.seed(seeds)
        eng.reset()
        P = eng.act_dim
        assert P == 50890
        rs = np.random.RandomState(21)
        for t in range(42):
            acts = rs.normal(0, 1e-3, (len(seeds), P)).astype(np.float32)
            out = eng.step(acts)
            for i, env in enumerate(refs):
                obs, reward, done, info = env.step(acts[i])
                if done:
                    obs = env.reset()
                assert bool(out['done'][i]) == done
                _row_close(out['obs'][i], obs)
                assert _rel(out['reward'][i], reward) <= RTOL
                assert _rel(out['objective'][i], info['objective']) <= RTOL
                assert out['accuracy'][i] == np.float32(info['accuracy'])
    finally:
        eng.close()


def test_config3_long_run_against_oracle():
    """205 steps of the fused config-3 kernel (five auto-resets): each reset
    composes the env's minibatch row order with its reset shuffle, so after
    five episodes every B = 32 minibatch still has to be the oracle's
    InMemoryDataSet rows (optimize.py:69-100, dataset/__init__.py); three
    envs against live oracle envs at every step."""
    from custom_envs_amd.data import load_data
    seq = load_data('mnist_synthetic', batch_size=32)
    seeds = [9, 10, 4000]
    eng = _engine(seq.features, seq.targets, len(seeds))
    refs = []
    for s in seeds:
        env = OracleEnv(seq.features, seq.targets, batch_size=32, model='mlp')
        env.seed(s)
        env.reset()
        refs.append(env)
    try:
        assert eng.step_kernel == 'mlp_step_kernel'
        eng.seed(seeds)
        eng.reset()
        P = eng.act_dim
        rs = np.random.RandomState(31)
        resets = 0
        for t in range(205):
            acts = rs.normal(0, 1e-3, (len(seeds), P)).astype(np.float32)
            out = eng.step(acts)
            for i, env in enumerate(refs):
                obs, reward, done, info = env.step(acts[i])
                if done:
                    obs = env.reset()
                    resets += 1
                what = 'env %d step %d' % (seeds[i], t)
                assert bool(out['done'][i]) == done, what
                assert int(out['episode_len'][i]) == info['episode']['l'], what
                _row_close(out['obs'][i], obs, what=what)
                assert _rel(out['reward'][i], reward) <= RTOL, what
                assert _rel(out['objective'][i], info['objective']) <= RTOL, what
                assert out['accuracy'][i] == np.float32(info['accuracy']), what
        assert resets == 3 * 5
        order = eng.get_state()['order']
        for i, env in enumerate(refs):
            assert np.array_equal(order[i], env.sequence.order), seeds[i]
    finally:
        eng.close()


def test_config3_benchmark_size_sampled_envs():
    """Config 3 at the size the bench runs it (BASELINE configs[2]: 4096
    envs, 784 -> 64 -> 10, N = 1024, B = 32): envs 0, 1, 2047, 2048, 4094 and
    4095 of the 4096-env grid against live oracle envs over 42 steps (one
    auto-reset), with device-resident actions and outputs as in bench.py."""
    import torch
    from custom_envs_amd.data import load_data
    seq = load_data('mnist_synthetic', batch_size=32)
    E = 4096
    sample = [0, 1, 2047, 2048, 4094, 4095]
    eng = _engine(seq.features, seq.targets, E)
    try:
        assert eng.step_kernel == 'mlp_step_kernel'
        eng.seed(list(range(E)))
        P = eng.act_dim
        out = eng.alloc_device_outputs()
        eng.reset_device(out)
        eng.wait()
        refs = []
        for s in sample:
            env = OracleEnv(seq.features, seq.targets, batch_size=32, model='mlp')
            env.seed(s)
            env.reset()
            refs.append(env)
        gen = torch.Generator(device='cuda')
        gen.manual_seed(1234)
        acts = torch.empty((E, P), dtype=torch.float32, device='cuda')
        idx = torch.tensor(sample, device='cuda')
        for t in range(42):
            acts.normal_(0.0, 1e-3, generator=gen)
            torch.cuda.synchronize()
            eng.step_device(acts, out)
            eng.wait()
            a = acts.index_select(0, idx).cpu().numpy()
            obs = out['obs'].view(E, -1).index_select(0, idx).cpu().numpy()
            got = {k: out[k].index_select(0, idx).cpu().numpy()
                   for k in ('reward', 'done', 'objective', 'accuracy', 'episode_len')}
            for i, env in enumerate(refs):
                o, reward, done, info = env.step(a[i])
                if done:
                    o = env.reset()
                what = 'env %d step %d' % (sample[i], t)
                assert bool(got['done'][i]) == done, what
                assert int(got['episode_len'][i]) == info['episode']['l'], what
                _row_close(obs[i], o, what=what)
                assert _rel(got['reward'][i], reward) <= RTOL, what
                assert _rel(got['objective'][i], info['objective']) <= RTOL, what
                assert got['accuracy'][i] == np.float32(info['accuracy']), what
    finally:
        eng.close()


def test_mlp_determinism_and_episode_cycle():
    from oracle.gen_golden import mlp_dataset
    features, targets = mlp_dataset()
    E = 300
    a = _engine(features, targets, E)
    b = _engine(features, targets, E)
    try:
        for eng in (a, b):
            eng.seed(list(range(100, 100 + E)))
        ra, rb = a.reset(), b.reset()
        assert not ra.any() and np.array_equal(ra, rb)
        rs = np.random.RandomState(8)
        for t in range(45):
            acts = rs.normal(0, 1e-3, (E, a.act_dim)).astype(np.float32)
            oa = {k: v.copy() for k, v in a.step(acts).items()}
            ob = b.step(acts)
            for k in oa:
                assert np.array_equal(oa[k], ob[k]), k
            assert np.all(oa['episode_len'] == t % 40 + 1)
            assert np.all(oa['done'] == (t % 40 == 39))
    finally:
        a.close()
        b.close()


def test_mlp_device_path_matches_host_path():
    import torch
    from oracle.gen_golden import mlp_dataset
    features, targets = mlp_dataset()
    E, K = 64, 12
    host = _engine(features, targets, E)
    dev = _engine(features, targets, E)
    try:
        for eng in (host, dev):
            eng.seed(list(range(E)))
        acts = np.random.RandomState(4).normal(0, 1e-3, (K, E, host.act_dim)).astype(np.float32)
        host.reset()
        for t in range(K):
            ref = host.step(acts[t])
        stream = torch.cuda.Stream()
        dev.set_stream(stream.cuda_stream)
        out = dev.alloc_device_outputs()
        with torch.cuda.stream(stream):
            a = torch.from_numpy(acts).cuda()
            stream.synchronize()
            dev.reset_device(out)
            dev.step_many_device(K, a, out)
            dev.wait()
        for k in ('obs', 'reward', 'done', 'objective', 'accuracy', 'episode_len'):
            np.testing.assert_array_equal(out[k].cpu().numpy(), ref[k], err_msg=k)
    finally:
        host.close()
        dev.close()


def test_make_optimize_mlp_env():
    from custom_envs_amd import make
    env = make('Optimize-v0', data_set='mnist_synthetic', batch_size=32, model='mlp')
    try:
        assert env.observation_space.shape == (2 * 50890 + 1,)
        assert env.action_space.shape == (50890,)
        env.seed(3)
        obs = env.reset()
        assert obs.shape == (101781,) and not obs.any()
        obs, reward, done, info = env.step(np.zeros(50890, np.float32))
        assert not done and set(info) == {'objective', 'accuracy', 'episode'}
        assert reward < 0 and info['episode']['l'] == 1
    finally:
        env.close()


@pytest.mark.parametrize('n_classes', [11, 10])
def test_odd_parameter_blocks_against_live_oracle(n_classes):
    """K = 11 makes P odd, so every odd env's parameter block starts at an odd
    float and takes the split pair accesses (mlp_kernels.h ld_f2/st_d2);
    F = 40 leaves a partial dW1 feature tile and a 5-chunk forward."""
    from oracle.gen_golden import mlp_dataset
    features, targets = mlp_dataset(n_rows=192, n_features=40, n_classes=n_classes)
    seeds = [3, 4, 5]
    eng = _engine(features, targets, len(seeds))
    refs = []
    for s in seeds:
        env = OracleEnv(features, targets, batch_size=32, model='mlp')
        env.seed(s)
        env.reset()
        refs.append(env)
    try:
        eng.seed(seeds)
        eng.reset()
        P = eng.act_dim
        assert P == 40 * 64 + 64 + 64 * n_classes + n_classes
        rs = np.random.RandomState(31)
        for t in range(43):
            acts = rs.normal(0, 1e-3, (len(seeds), P)).astype(np.float32)
            out = eng.step(acts)
            for i, env in enumerate(refs):
                obs, reward, done, info = env.step(acts[i])
                if done:
                    obs = env.reset()
                assert bool(out['done'][i]) == done
                _row_close(out['obs'][i], obs)
                assert _rel(out['reward'][i], reward) <= RTOL
                assert _rel(out['objective'][i], info['objective']) <= RTOL
                assert out['accuracy'][i] == np.float32(info['accuracy'])
            if not out['done'].any():
                w = eng.get_state()['weights'].astype(np.float32)
                for i, env in enumerate(refs):
                    assert np.array_equal(w[i], env.model.weights.astype(np.float32)), (t, i)
    finally:
        eng.close()


def test_fused_step_matches_split_kernels(monkeypatch):
    """mlp_step_kernel (one launch) and the split train + info pair run the
    same arithmetic: bit-identical outputs, except the objective, whose
    per-wave partial sums cover different tile sets (4 vs 8 tiles per pass)."""
    from oracle.gen_golden import mlp_dataset
    features, targets = mlp_dataset(n_rows=256, n_features=64)
    E = 37
    fused = _engine(features, targets, E)
    monkeypatch.setenv('CE_MLP_SPLIT', '1')
    split = _engine(features, targets, E)
    try:
        assert fused.step_kernel == 'mlp_step_kernel'
        assert split.step_kernel == 'mlp_train_kernel+mlp_info_kernel'
        for eng in (fused, split):
            eng.seed(list(range(E)))
            eng.reset()
        rs = np.random.RandomState(5)
        for t in range(41):
            acts = rs.normal(0, 1e-3, (E, fused.act_dim)).astype(np.float32)
            a = {k: v.copy() for k, v in fused.step(acts).items()}
            b = split.step(acts)
            for k in a:
                if k == 'objective':
                    np.testing.assert_allclose(a[k], b[k], rtol=1e-6, err_msg=str(t))
                else:
                    assert np.array_equal(a[k], b[k]), (t, k)
    finally:
        fused.close()
        split.close()


# ---------------------------------------------------------------------------
# The layered network path (net_engine.hip): Optimize-v0 over any OptimizeNN
# network (create_neural_net's default (256, 256), optimize_nn.py:22-64,
# utils_tf.py:74-86) and any batch size.  Same tolerances as above; accuracy
# may differ by one row where two float32 probabilities tie to rounding.

def _net_engine(features, targets, num_envs, hidden, batch_size, monkeypatch=None, force=False):
    from custom_envs_amd.engine import OptimizeEngine
    if force:
        monkeypatch.setenv('CE_MLP_NET', '1')
    eng = OptimizeEngine(features, targets, num_envs=num_envs, batch_size=batch_size, model='mlp',
                         hidden=hidden)
    if force:
        monkeypatch.delenv('CE_MLP_NET')
    return eng


def _relu_ties(model, weights, X, rel=2e-6):
    """The hidden pre-activations of this minibatch that lie within float32
    rounding of zero (|z| < rel * (sum_k |x_k w_k| + |b|)), as (layer, sample,
    unit) triples: the two float32 evaluations (numpy and the engine's GEMMs,
    summing in different orders) may take different sides of the relu kink
    there, which moves the gradient by that sample's term through that
    unit."""
    h = np.asarray(X, np.float32)
    start = 0
    dims = model.dims
    ties = []
    for layer, (din, dout) in enumerate(zip(dims[:-2], dims[1:-1])):
        w = weights[start:start + din * dout].reshape(din, dout)
        b = weights[start + din * dout:start + din * dout + dout]
        start += din * dout + dout
        z = h @ w + b
        mag = np.abs(h) @ np.abs(w) + np.abs(b)
        ties += [(layer, int(s), int(u)) for s, u in zip(*np.nonzero(np.abs(z) < rel * mag))]
        h = np.maximum(z, 0)
    return ties


def _tie_variant_rows(model, weights, X, Y, g_prev, l_new, ties):
    """Observation rows [0 | L' | (g / B) / (|G| + 1)] of the oracle's float32
    backward with the relu masks of every subset of the tied units flipped
    (the forward is unchanged to within |z|, far below the tolerance)."""
    w_all = np.asarray(weights, np.float32)
    dims = model.dims
    kernels, biases, start = [], [], 0
    for din, dout in zip(dims[:-1], dims[1:]):
        kernels.append(w_all[start:start + din * dout].reshape(din, dout))
        start += din * dout
        biases.append(w_all[start:start + dout])
        start += dout
    acts, pre = [np.asarray(X, np.float32)], []
    for w, b in zip(kernels[:-1], biases[:-1]):
        z = acts[-1] @ w + b
        pre.append(z)
        acts.append(np.maximum(z, np.float32(0)))
    from oracle.optimize import softmax
    prob = softmax(acts[-1] @ kernels[-1] + biases[-1])
    rows = []
    for bits in range(1 << len(ties)):
        masks = [(z > 0) for z in pre]
        for k, (layer, s, u) in enumerate(ties):
            if bits >> k & 1:
                masks[layer][s, u] = not masks[layer][s, u]
        dz = prob - np.asarray(Y, np.float32)
        grads = []
        for layer in range(len(kernels) - 1, -1, -1):
            grads = [(acts[layer].T @ dz).ravel(), dz.sum(axis=0)] + grads
            if layer > 0:
                dz = (dz @ kernels[layer].T) * masks[layer - 1]
        g = np.concatenate(grads) / np.float32(len(X))
        gn = g.astype(np.float64) / (np.abs(g_prev) + 1)
        rows.append(np.concatenate([np.zeros(model.size), [l_new], gn]))
    return rows


def _net_check(features, targets, eng, hidden, batch_size, seeds, steps, scale=1e-3):
    """Tolerances as for config 3.  At a step whose minibatch has relu ties
    (_relu_ties) the observation row must match, within the same tolerance,
    the oracle's row for SOME choice of sides at the tied units
    (_tie_variant_rows; up to 4 ties, else at most 0.5 % of the row's entries
    may exceed the tolerance); the reward / objective checks stay exact."""
    refs = []
    for s in seeds:
        env = OracleEnv(features, targets, batch_size=batch_size, model='mlp', hidden=hidden)
        env.seed(s)
        env.reset()
        refs.append(env)
    eng.seed(seeds)
    assert np.all(eng.reset() == 0)
    P = eng.act_dim
    assert P == refs[0].model.size
    n_rows = len(features)
    rs = np.random.RandomState(len(seeds) + P)
    ties = 0
    for t in range(steps):
        acts = rs.normal(0, scale, (len(seeds), P)).astype(np.float32)
        out = eng.step(acts)
        st = eng.get_state()
        weights = st['weights'].astype(np.float32)
        for i, env in enumerate(refs):
            w_new = env.model.weights - acts[i]
            X, Y = env.sequence[0]
            tie = _relu_ties(env.model, w_new, X)
            g_prev = env.grad_hist[env.current_step % 3].ravel().copy()
            obs, reward, done, info = env.step(acts[i])
            if not done:     # W <- W - a is one float32 subtraction on both sides
                assert np.array_equal(weights[i], env.model.weights), (i, t)
            if done:
                obs = env.reset()
            assert bool(out['done'][i]) == done, (i, t)
            assert int(out['episode_len'][i]) == info['episode']['l']
            assert not out['obs'][i][:P].any()
            if tie and not done:
                ties += 1
                if len(tie) <= 4:
                    rows = _tie_variant_rows(env.model, w_new, X, Y, g_prev, obs[P], tie)
                    assert np.allclose(rows[0], obs, rtol=0, atol=1e-12 + 1e-6 * np.abs(obs).max())
                    errs = []
                    for k, row in enumerate(rows):
                        try:
                            _row_close(out['obs'][i], row, what='env %d step %d' % (i, t))
                            break
                        except AssertionError as exc:
                            errs.append(str(exc))
                    else:
                        raise AssertionError('no side choice of %d relu ties matches: %s'
                                             % (len(tie), errs[0]))
                    if k:    # the engine took the other side: follow its gradient history
                        env.grad_hist[env.current_step % 3] = st['grad_hist'][i]
                else:
                    scale_r = max(np.abs(obs).max(), 1e-30)
                    bad = np.abs(out['obs'][i].astype(np.float64) - obs) > RTOL * scale_r
                    assert bad.mean() <= 5e-3, (i, t, int(bad.sum()))
            else:
                _row_close(out['obs'][i], obs, what='env %d step %d' % (i, t))
            assert _rel(out['reward'][i], reward) <= RTOL, (i, t)
            assert _rel(out['objective'][i], info['objective']) <= RTOL, (i, t)
            assert abs(float(out['accuracy'][i]) - info['accuracy']) <= 1.5 / n_rows, (i, t)
    return ties


@pytest.mark.parametrize('batch_size', [16, 32, 100])
def test_default_network_256x256(batch_size):
    """create_neural_net's default layers (256, 256) over the MNIST-sized set
    (1024 x 784, 10 classes): P = 269,322; 3 envs across an auto-reset; B of
    16, 32 and 100 (a batch that is not a multiple of anything)."""
    from custom_envs_amd.data import load_data
    seq = load_data('mnist_synthetic', batch_size=batch_size)
    eng = _net_engine(seq.features, seq.targets, 3, (256, 256), batch_size)
    try:
        assert eng.step_kernel == 'net<784,256,256,10>:mfma'   # the hand-written MFMA kernels
        _net_check(seq.features, seq.targets, eng, (256, 256), batch_size, [3, 4, 5], 42)
    finally:
        eng.close()


@pytest.mark.parametrize('hidden,batch_size', [((96, 32, 48), 20), ((40,), None), ((64,), 32),
                                               ((33, 7), 24)])
def test_network_shapes(hidden, batch_size, monkeypatch):
    """Three hidden layers, one layer with the full batch (B = N: the info pass
    reuses the minibatch numbers), config 3's shape forced onto the layered
    path (CE_MLP_NET=1), and odd widths (P = 26,223 is odd: the epilogue's
    scalar path, bias slabs off 8-byte boundaries) -- 5 envs, one
    mid-episode reset crossed."""
    from oracle.gen_golden import mlp_dataset
    features, targets = mlp_dataset()
    force = hidden == (64,)
    eng = _net_engine(features, targets, 5, hidden, batch_size, monkeypatch, force=force)
    try:
        assert eng.step_kernel.startswith('net<')
        _net_check(features, targets, eng, hidden, batch_size, [7, 8, 9, 10, 11], 43, scale=3e-3)
    finally:
        eng.close()


@pytest.mark.parametrize('n_classes', [16, 17, 32])
def test_network_class_counts(n_classes):
    """The output layer's two forward forms at their boundary: up to 16
    classes one MFMA block per K step (net_layer_narrow, the softmax
    gathering class 4g + i from lane group g), 17 to 32 the four-block form
    -- 3 envs, 41 steps across an auto-reset."""
    from oracle.gen_golden import mlp_dataset
    features, targets = mlp_dataset(n_rows=192, n_features=40, n_classes=n_classes)
    eng = _net_engine(features, targets, 3, (64, 48), 24)
    try:
        assert eng.step_kernel.endswith(':mfma')
        _net_check(features, targets, eng, (64, 48), 24, [4, 5, 6], 41, scale=3e-3)
    finally:
        eng.close()


@pytest.mark.parametrize('hidden,batch_size', [((300,), 24), ((260, 300), None), ((512, 40, 33), 32)])
def test_wide_network_against_oracle(hidden, batch_size):
    """Hidden layers wider than 256 units (create_neural_net accepts any
    width, utils/utils_model.py:34): the wide-layer path (net_wide.h, a
    natural weight image, tiled float32 kernels; the gradient's float64
    epilogue and the finish kernel shared with the MFMA path) against the
    oracle -- a minibatch, the full batch (B = N), three hidden layers with
    odd widths; 3 envs across an auto-reset, weights bit-equal every step."""
    from oracle.gen_golden import mlp_dataset
    features, targets = mlp_dataset()
    eng = _net_engine(features, targets, 3, hidden, batch_size)
    try:
        assert eng.step_kernel == 'net<%s>:wide' % ','.join(map(str, (16,) + hidden + (10,)))
        _net_check(features, targets, eng, hidden, batch_size, [21, 22, 23], 41, scale=3e-3)
    finally:
        eng.close()


def test_wide_network_many_envs():
    """The wide path's grids at more envs than tiles (the GEMM's z
    dimension, the loss tiles, the grad kernel's XCD walk): 70 envs of
    16 -> 300 -> 10, B = 24, every env against its oracle over 41 steps."""
    from oracle.gen_golden import mlp_dataset
    features, targets = mlp_dataset()
    eng = _net_engine(features, targets, 70, (300,), 24)
    try:
        assert eng.step_kernel == 'net<16,300,10>:wide'
        _net_check(features, targets, eng, (300,), 24, list(range(100, 170)), 41, scale=3e-3)
    finally:
        eng.close()


def test_wide_network_512_on_mnist_shape():
    """an oracle test at width 512 -- 784 -> 512 -> 10 over the
    MNIST-sized set (1024 x 784), B = 32, 2 envs across an auto-reset; and the
    state round trip through the natural image (set_state / get_state)."""
    from custom_envs_amd.data import load_data
    seq = load_data('mnist_synthetic', batch_size=32)
    eng = _net_engine(seq.features, seq.targets, 2, (512,), 32)
    try:
        assert eng.step_kernel == 'net<784,512,10>:wide'
        _net_check(seq.features, seq.targets, eng, (512,), 32, [5, 6], 41)
        st = eng.get_state()
        rs = np.random.RandomState(1)
        w = rs.normal(0, 0.05, st['weights'].shape).astype(np.float32).astype(np.float64)
        eng.set_state(weights=w)
        assert np.array_equal(eng.get_state()['weights'], w)
    finally:
        eng.close()


def test_network_full_batch_and_depth():
    """The default network with the full batch (B = N: every row is a
    minibatch row, the info numbers are the minibatch's), and three hidden
    layers with a minibatch -- the shapes the rocBLAS arm used to cover."""
    from oracle.gen_golden import mlp_dataset
    features, targets = mlp_dataset()
    for hidden, batch_size in (((96, 32, 48), 20), ((256, 256), None)):
        eng = _net_engine(features, targets, 3, hidden, batch_size)
        try:
            assert eng.step_kernel.endswith(':mfma')
            _net_check(features, targets, eng, hidden, batch_size, [7, 8, 9], 41, scale=3e-3)
        finally:
            eng.close()


def test_network_state_roundtrip():
    """ce_set_state / ce_get_state through the weight images (net_kernels.h):
    the flat [W1 | b1 | ...] vector comes back bit for bit, odd widths
    included, and a step from a set state matches the oracle."""
    from oracle.gen_golden import mlp_dataset
    features, targets = mlp_dataset()
    for hidden in ((33, 7), (256, 256)):
        eng = _net_engine(features, targets, 2, hidden, 24)
        try:
            eng.seed([1, 2])
            eng.reset()
            st = eng.get_state()
            rs = np.random.RandomState(5)
            w = rs.normal(0, 0.1, st['weights'].shape).astype(np.float32).astype(np.float64)
            eng.set_state(weights=w, init_weights=w[::-1].copy())
            back = eng.get_state()
            assert np.array_equal(back['weights'], w)
            assert np.array_equal(back['init_weights'], w[::-1])
            # a row order written by set_state moves the minibatch (its slots)
            perms = np.stack([rs.permutation(len(features)) for _ in range(2)]).astype(np.int32)
            eng.set_state(order=perms)
            assert np.array_equal(eng.get_state()['order'], perms)
            acts = rs.normal(0, 1e-3, w.shape).astype(np.float32)
            out = eng.step(acts)
            from oracle.optimize import ModelMLP
            for i in range(2):
                model = ModelMLP(features.shape[1], targets.shape[1], hidden)
                model.set_weights(w[i].astype(np.float32) - acts[i])
                rows = perms[i][:24]
                loss, grad, _ = model.compute_backprop(features[rows].astype(np.float32),
                                                       targets[rows].astype(np.float32))
                assert _rel(out['reward'][i], -loss) <= RTOL, (hidden, i)
                gn = (grad / np.float32(24)).astype(np.float64) / (np.abs(back['grad_hist'][i]) + 1)
                P = w.shape[1]
                _row_close(out['obs'][i], np.concatenate([np.zeros(P), [out['obs'][i][P]], gn]),
                           what='set_state order %s env %d' % (hidden, i))
        finally:
            eng.close()


def test_network_seed_draws_match_numpy():
    """W0 of a two-layer network: glorot-uniform per layer then the reset
    shuffle on the same stream (oracle.initial_draws_mlp)."""
    from custom_envs_amd.data import load_data
    from oracle.optimize import initial_draws_mlp
    seq = load_data('mnist_synthetic', batch_size=32)
    eng = _net_engine(seq.features, seq.targets, 2, (256, 256), 32)
    try:
        eng.seed([11, 12])
        eng.reset()
        st = eng.get_state()
        for i, s in enumerate((11, 12)):
            w0, perm = initial_draws_mlp(s, 784, (256, 256), 10, 1024)
            assert np.array_equal(st['init_weights'][i].astype(np.float32), w0)
            assert np.array_equal(st['order'][i], perm)
    finally:
        eng.close()
