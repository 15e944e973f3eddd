"""Regenerate the committed golden fixtures under tests/golden/.

Run from the repo root:  python -m oracle.gen_golden
The fixtures are data (inputs + expected outputs of the oracle); the
dataset fixture is the source of truth for every config using the 256x10
logistic-regression problem.
"""
import os

import numpy as np

from oracle.data import gaussians
from oracle.optimize import Optimize, initial_draws
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


def main():
    os.makedirs(GOLDEN, exist_ok=True)
    features, targets = write_dataset()
    write_seeding(features)
    write_rollouts(features, targets)


if __name__ == '__main__':
    main()
