"""Episode logging: the scripts' ``Monitor`` and a vectorised ``VecMonitor``.

``Monitor`` keeps the reference's constructor and behaviour
(custom_envs/utils/utils_logging.py:15-156): callbacks fed every step,
episode rows ``r, l, t, current_reward, episode`` plus ``info_keywords``
appended on done and written in ``chunk_size`` chunks to ``<path>.mon.csv``
with sorted columns.  Two reference bugs are not reproduced:
``get_total_steps`` counts steps (the reference reads an attribute it never
sets) and ``get_episode_times`` returns times (the reference returns rewards).

``VecMonitor`` does the same bookkeeping for a whole engine-backed vector env
from its batched reward/done arrays, so monitored envs do not put a Python
wrapper call per env per step back on the hot path.
"""
import time
from collections import defaultdict
from pathlib import Path

import numpy as np

from custom_envs_amd.core import Wrapper

EXT = '.mon.csv'


def _mon_path(file_path):
    return None if file_path is None else Path(file_path).resolve().with_suffix(EXT)


def _save_rows(path, rows):
    if path is None or not rows:
        return
    import pandas as pd
    header = not path.is_file()
    frame = pd.DataFrame(rows)
    frame = frame.reindex(sorted(frame.columns), axis=1)
    frame.to_csv(path, header=header, index=False, mode='w' if header else 'a')


class Monitor(Wrapper):
    """utils_logging.Monitor: wraps one env (or an env factory)."""
    EXT = EXT

    def __init__(self, env, file_path, info_keywords=(), chunk_size=1, callbacks=None,
                 allow_early_resets=True):
        if callable(env) and not hasattr(env, 'step'):
            env = env()
        super().__init__(env)
        self.t_start = time.time()
        self.file_path = _mon_path(file_path)
        self.chunk_size = chunk_size
        self.info_keywords = info_keywords
        self.allow_early_resets = allow_early_resets
        self.last_info = {}
        self.rewards = None
        self.metric_history = defaultdict(list)
        self.current_episode = 0
        self.callbacks = [] if callbacks is None else callbacks
        self.data = []
        self.total_steps = 0

    def save(self):
        _save_rows(self.file_path, self.data)
        self.data = []

    def reset(self, **kwargs):
        self.rewards = []
        self.current_episode += 1
        return self.env.reset(**kwargs)

    def step(self, action):
        observation, reward, done, info = self.env.step(action)
        for callback in self.callbacks:
            callback({'observation': observation, 'reward': reward, 'done': done,
                      'info': info, 'episode': self.current_episode})
        self.rewards.append(reward)
        self.total_steps += 1
        if done:
            ep_rew = sum(self.rewards)
            ep_info = {'r': round(ep_rew, 6), 'l': len(self.rewards),
                       't': round(time.time() - self.t_start, 6),
                       'current_reward': reward, 'episode': self.current_episode}
            self.last_info = info
            for key in self.info_keywords:
                ep_info[key] = info[key]
            self.data.append(ep_info)
            if len(self.data) >= self.chunk_size:
                self.save()
            info['episode'] = ep_info
            self.metric_history['rewards'].append(ep_rew)
            self.metric_history['lengths'].append(len(self.rewards))
            self.metric_history['times'].append(time.time() - self.t_start)
        return observation, reward, done, info

    def close(self):
        if self.data:
            self.save()
        return self.env.close()

    def get_total_steps(self):
        return self.total_steps

    def get_episode_rewards(self):
        return self.metric_history.get('rewards', [])

    def get_episode_lengths(self):
        return self.metric_history.get('lengths', [])

    def get_episode_times(self):
        return self.metric_history.get('times', [])


class VecMonitor:
    """Monitor bookkeeping for E envs at once (one row of arrays per step).

    ``file_paths`` is one path (or None) per env, as the per-env Monitors of
    the reference had; ``step`` takes per-env rewards, dones and an info
    sequence and returns the per-env episode dicts of envs that finished.
    ``style``: 'logging' writes utils_logging.Monitor's rows (r, l, t,
    current_reward, episode + info_keywords; utils_logging.py:98-116),
    'sb' the stable-baselines wrappers.monitor.Monitor's (r, l, t +
    info_keywords, monitor.py:94-123), whose reset refuses envs still in an
    episode unless ``allow_early_resets`` (monitor.py:69-75).
    """

    def __init__(self, num_envs, file_paths=None, info_keywords=(), chunk_size=1,
                 callbacks=None, style='logging', allow_early_resets=True,
                 reset_keywords=()):
        if style not in ('logging', 'sb'):
            raise ValueError('style must be logging or sb')
        self.style = style
        self.reset_keywords = tuple(reset_keywords or ())
        if self.reset_keywords and style != 'sb':
            raise ValueError('reset_keywords belong to the sb style')
        self.allow_early_resets = bool(allow_early_resets)
        self.needs_reset = np.ones(num_envs, bool)
        self.num_envs = num_envs
        if file_paths is None or isinstance(file_paths, (str, Path)):
            file_paths = [file_paths] * num_envs if file_paths is None else [
                '%s_%d' % (file_paths, i) for i in range(num_envs)]
        self.paths = [_mon_path(p) for p in file_paths]
        self.info_keywords = tuple(info_keywords)
        self.chunk_size = chunk_size
        self.callbacks = list(callbacks or ())
        self.t_start = time.time()
        self.ep_reward = np.zeros(num_envs)
        self.ep_len = np.zeros(num_envs, np.int64)
        self.current_episode = np.zeros(num_envs, np.int64)
        self.data = [[] for _ in range(num_envs)]
        self.metric_history = [defaultdict(list) for _ in range(num_envs)]
        self.total_steps = np.zeros(num_envs, np.int64)
        # per env, as each reference Monitor keeps its own current_reset_info
        # (monitor.py:84-90): a partial reset stamps only the envs it resets
        self.reset_info = [{} for _ in range(num_envs)]

    def reset(self, indices=None, **kwargs):
        idx = slice(None) if indices is None else indices
        if self.style == 'sb' and not self.allow_early_resets and not self.needs_reset[idx].all():
            raise RuntimeError('Tried to reset an environment before done. If you want to '
                               'allow early resets, wrap your env with Monitor(env, path, '
                               'allow_early_resets=True)')
        self.needs_reset[idx] = False         # before the keyword check, monitor.py:84-85
        for key in self.reset_keywords:
            if kwargs.get(key) is None:
                raise ValueError('Expected you to pass kwarg %s into reset' % key)
        envs = range(len(self.reset_info)) if indices is None else np.arange(
            len(self.reset_info))[indices]
        for i in np.atleast_1d(envs):
            for key in self.reset_keywords:
                self.reset_info[int(i)][key] = kwargs[key]
        self.ep_reward[idx] = 0.0
        self.ep_len[idx] = 0
        self.current_episode[idx] += 1

    def check_step(self):
        """Called before the engine launches a step: the SB Monitor refuses
        to step an env that needs a reset (monitor.py:87-88)."""
        if self.style == 'sb' and self.needs_reset.any():
            raise RuntimeError('Tried to step environment that needs reset')

    def step(self, rewards, dones, infos, observations=None):
        rewards = np.asarray(rewards, dtype=np.float64)
        dones = np.asarray(dones, dtype=bool)
        if self.callbacks:
            for i in range(self.num_envs):
                payload = {'observation': None if observations is None else observations[i],
                           'reward': float(rewards[i]), 'done': bool(dones[i]),
                           'info': infos[i], 'episode': int(self.current_episode[i])}
                for callback in self.callbacks:
                    callback(payload)
        self.ep_reward += rewards
        self.ep_len += 1
        self.total_steps += 1
        finished = {}
        now = time.time() - self.t_start
        for i in np.flatnonzero(dones):
            info = infos[i]
            self.needs_reset[i] = True
            ep_info = {'r': round(float(self.ep_reward[i]), 6), 'l': int(self.ep_len[i]),
                       't': round(now, 6)}
            if self.style == 'logging':
                ep_info['current_reward'] = float(rewards[i])
                ep_info['episode'] = int(self.current_episode[i])
            for key in self.info_keywords:
                ep_info[key] = info[key]
            ep_info.update(self.reset_info[i])
            self.data[i].append(ep_info)
            if len(self.data[i]) >= self.chunk_size:
                _save_rows(self.paths[i], self.data[i])
                self.data[i] = []
            history = self.metric_history[i]
            history['rewards'].append(float(self.ep_reward[i]))
            history['lengths'].append(int(self.ep_len[i]))
            history['times'].append(now)
            finished[int(i)] = ep_info
        if finished:   # auto-reset happened in the engine: the Monitor's reset()
            self.reset(list(finished))
        return finished

    def close(self):
        for i in range(self.num_envs):
            _save_rows(self.paths[i], self.data[i])
            self.data[i] = []

    def get_episode_rewards(self, indices=None):
        idx = range(self.num_envs) if indices is None else indices
        return [self.metric_history[i].get('rewards', []) for i in idx]

    def get_episode_lengths(self, indices=None):
        idx = range(self.num_envs) if indices is None else indices
        return [self.metric_history[i].get('lengths', []) for i in idx]

    def get_episode_times(self, indices=None):
        idx = range(self.num_envs) if indices is None else indices
        return [self.metric_history[i].get('times', []) for i in idx]

    def get_total_steps(self, indices=None):
        idx = range(self.num_envs) if indices is None else indices
        return [int(self.total_steps[i]) for i in idx]


def create_env(env_name, log_dir=None, num_of_envs=1, **kwargs):
    """utils_logging.py:159-175."""
    from custom_envs_amd.core import make
    envs = [make(env_name, **kwargs) for _ in range(num_of_envs)]
    if log_dir is not None:
        log_dir = Path(log_dir)
        envs = [Monitor(env, str(log_dir / str(i)), chunk_size=10,
                        info_keywords=('objective', 'accuracy'))
                for i, env in enumerate(envs)]
    return envs
