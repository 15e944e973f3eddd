"""Regenerate the committed golden fixtures under tests/golden/.

Run from the repo root:  python -m oracle.gen_golden
The fixtures are data (inputs + expected outputs of the oracle); the
dataset fixture is the source of truth for every config using the 256x10
logistic-regression problem.
"""
import os

import numpy as np

from oracle.data import gaussians
from oracle.optimize import Optimize, initial_draws, initial_draws_mlp
from oracle.seeding import seed_key

HERE = os.path.dirname(os.path.abspath(__file__))
GOLDEN = os.path.join(HERE, os.pardir, 'tests', 'golden')

SEEDS = (0, 1, 2, 7, 1023, 4095, 123456789, 2**32 + 5, 2**63 + 11)


def write_dataset():
    features, targets = gaussians(256, 10, 0)
    np.savez_compressed(os.path.join(GOLDEN, 'lr_256x10.npz'),
                        features=features, targets=targets)
    return features, targets


def write_seeding(features):
    n_rows, n_features = features.shape
    keys = np.zeros((len(SEEDS), 3), np.int64)
    key_len = np.zeros(len(SEEDS), np.int64)
    weights = np.zeros((len(SEEDS), n_features, 2))
    perms = np.zeros((len(SEEDS), n_rows), np.int64)
    for i, seed in enumerate(SEEDS):
        key = seed_key(seed)
        keys[i, :len(key)] = key
        key_len[i] = len(key)
        weights[i], perms[i] = initial_draws(seed, n_features, 2, n_rows)
    # odd draw count (F*K = 3*3 = 9) exercises the cached-gaussian slot
    w_odd, p_odd = initial_draws(5, 3, 3, 150)
    np.savez_compressed(os.path.join(GOLDEN, 'seeding.npz'),
                        seeds=np.array(SEEDS, dtype=np.uint64), keys=keys,
                        key_len=key_len, weights=weights, perms=perms,
                        w_odd=w_odd, p_odd=p_odd)


def rollout(features, targets, seed, batch_size, steps, action_seed):
    env = Optimize(features, targets, batch_size=batch_size)
    env.seed(seed)
    n_params = env.model.size
    actions = np.random.RandomState(action_seed).normal(
        0, 0.01, (steps, n_params)).astype(np.float32)
    first = env.reset()
    rec = {k: [] for k in ('obs', 'reward', 'done', 'objective', 'accuracy',
                           'ep_len', 'order', 'weights')}
    for t in range(steps):
        obs, reward, done, info = env.step(actions[t])
        rec['ep_len'].append(info['episode']['l'])
        if done:                      # VecEnv auto-reset (utils_venv.py:31)
            obs = env.reset()
        rec['obs'].append(obs)
        rec['reward'].append(reward)
        rec['done'].append(done)
        rec['objective'].append(info['objective'])
        rec['accuracy'].append(info['accuracy'])
        rec['order'].append(env.sequence.order.copy())
        rec['weights'].append(env.model.weights.ravel().copy())
    out = {k: np.array(v) for k, v in rec.items()}
    out['actions'] = actions
    out['reset_obs'] = first
    out['seed'] = np.array(seed)
    out['batch_size'] = np.array(-1 if batch_size is None else batch_size)
    return out


def write_rollouts(features, targets):
    for seed in (0, 1, 2):
        rec = rollout(features, targets, seed, None, 45, 1234 + seed)
        del rec['order']               # B == N: the order never matters
        np.savez_compressed(
            os.path.join(GOLDEN, 'optimize_lr_s%d.npz' % seed), **rec)
    for seed in (3, 4):
        rec = rollout(features, targets, seed, 32, 85, 99 + seed)
        np.savez_compressed(
            os.path.join(GOLDEN, 'optimize_lr_b32_s%d.npz' % seed), **rec)


def rollout_multi(ndims, max_batches, max_history, steps, action_seed, low=1.0, high=3.0):
    """OptVecEnv semantics around one MultiOptLRs env: rows in sorted agent
    order, auto-reset on done (optvecenv.py:38-46, concurrentvecenv.py:37)."""
    from oracle.multioptlrs import MultiOptLRs, OptEnvRunner
    env = MultiOptLRs(ndims, max_batches=max_batches, max_history=max_history)
    runner = OptEnvRunner(env)
    rs = np.random.RandomState(action_seed)
    first = np.stack(runner.reset())
    keys = ('loss', 'batch_loss', 'weights_mean', 'weights_sum', 'actions_mean', 'actions_std',
            'states_mean', 'states_sum', 'grads_mean', 'grads_sum', 'loss_mean',
            'adjusted_loss', 'adjusted_grad', 'grad_diff')
    rec = {k: [] for k in ('obs', 'reward', 'done', 'info', 'ep_len', 'theta')}
    actions = rs.uniform(low, high, (steps, ndims, 1)).astype(np.float32)
    for t in range(steps):
        states, rewards, dones, infos = runner.step(list(actions[t]))
        info = infos[0]
        rec['ep_len'].append(info['episode']['l'])
        rec['info'].append([np.nan if info[k] is None else float(info[k]) for k in keys])
        rec['theta'].append(env.model.params.copy())
        if any(dones):
            states = runner.reset()
        rec['obs'].append(np.stack(states))
        rec['reward'].append(rewards[0])
        rec['done'].append(dones[0])
    out = {k: np.array(v) for k, v in rec.items()}
    out['actions'] = actions
    out['reset_obs'] = first
    return out


MLP_KEEP = (0, 1, 19, 39, 40, 44)      # steps whose full obs / weights are stored


def mlp_dataset(n_rows=128, n_features=16, n_classes=10):
    """Small MLP fixture problem: uniform features, argmax((X - 1/2) T) labels."""
    features = np.random.RandomState(2).rand(n_rows, n_features)
    proj = np.random.RandomState(3).normal(size=(n_features, n_classes))
    targets = np.eye(n_classes)[np.argmax((features - 0.5) @ proj, axis=1)]
    return features, targets


def mlp_actions(action_seed, steps, n_params):
    return np.random.RandomState(action_seed).normal(0, 1e-3, (steps, n_params)).astype(
        np.float32)


def rollout_mlp(features, targets, seed, steps=45, action_seed=77, hidden=64):
    """Optimize over the A12 MLP, B = 32, VecEnv auto-reset (utils_venv.py:31)."""
    env = Optimize(features, targets, batch_size=32, model='mlp', hidden=hidden)
    env.seed(seed)
    first = env.reset()
    P = env.model.size
    actions = mlp_actions(action_seed, steps, P)
    rec = {k: [] for k in ('reward', 'done', 'objective', 'accuracy', 'ep_len', 'loss_obs',
                           'obs', 'weights')}
    for t in range(steps):
        obs, reward, done, info = env.step(actions[t])
        rec['ep_len'].append(info['episode']['l'])
        weights = env.model.weights.copy()
        if done:
            obs = env.reset()
        rec['reward'].append(reward)
        rec['done'].append(done)
        rec['objective'].append(info['objective'])
        rec['accuracy'].append(info['accuracy'])
        rec['loss_obs'].append(obs[P])
        if t in MLP_KEEP:
            rec['obs'].append(obs.astype(np.float32))
            rec['weights'].append(weights)
    out = {k: np.array(v) for k, v in rec.items()}
    out['reset_obs'] = first.astype(np.float32)
    out['init_weights'] = initial_draws_mlp(seed, features.shape[1], hidden,
                                            targets.shape[1], len(features))[0]
    out['seed'] = np.array(seed)
    out['action_seed'] = np.array(action_seed)
    out['keep'] = np.array(MLP_KEEP)
    return out


def write_mlp():
    features, targets = mlp_dataset()
    np.savez_compressed(os.path.join(GOLDEN, 'mlp_data_128x16.npz'), features=features,
                        targets=targets)
    for seed in (5, 6):
        rec = rollout_mlp(features, targets, seed, action_seed=77 + seed)
        np.savez_compressed(os.path.join(GOLDEN, 'optimize_mlp_s%d.npz' % seed), **rec)


def write_multi():
    # (name, ndims, max_batches, max_history, steps, seed, action range):
    # stable learning rates (10^-5..10^-3.5), the configs' 10^-3..10^-1
    # (diverges: loss > 1e4 early stop), and a mix hitting max_batches
    cases = [('multi_func2_h5', 2, 400, 5, 150, 7, -1.0, 0.5),
             ('multi_func4_h5', 4, 400, 5, 60, 8, 1.0, 3.0),
             ('multi_func4_h3_b25', 4, 25, 3, 90, 9, -1.0, 0.7)]
    for name, ndims, max_batches, hist, steps, seed, low, high in cases:
        rec = rollout_multi(ndims, max_batches, hist, steps, seed, low, high)
        np.savez_compressed(os.path.join(GOLDEN, name + '.npz'), **rec)


def main():
    os.makedirs(GOLDEN, exist_ok=True)
    features, targets = write_dataset()
    write_seeding(features)
    write_rollouts(features, targets)
    write_multi()
    write_mlp()


if __name__ == '__main__':
    main()
