"""Stable-baselines style Monitor (custom_envs/wrappers/monitor.py:11-163).

Differs from ``utils.utils_logging.Monitor`` by the SB contract: reset is
refused before an episode ends unless ``allow_early_resets``, stepping a
finished env is refused, ``reset_keywords`` are required reset kwargs whose
values are logged, and the episode row has ``r, l, t`` plus
``info_keywords``.
"""
import time

from custom_envs_amd.core import Wrapper
from custom_envs_amd.utils.utils_logging import EXT, _mon_path, _save_rows


class Monitor(Wrapper):
    EXT = EXT

    def __init__(self, env, file_path, allow_early_resets=False, reset_keywords=(),
                 info_keywords=(), chunk_size=1):
        super().__init__(env)
        self.t_start = time.time()
        self.file_path = _mon_path(file_path)
        self.chunk_size = chunk_size
        self.reset_keywords = reset_keywords
        self.info_keywords = info_keywords
        self.allow_early_resets = allow_early_resets
        self.rewards = None
        self.needs_reset = True
        self.episode_rewards, self.episode_lengths, self.episode_times = [], [], []
        self.total_steps = 0
        self.current_reset_info = {}
        self.data = []

    def save(self):
        _save_rows(self.file_path, self.data)
        self.data = []

    def reset(self, **kwargs):
        if not self.allow_early_resets and not self.needs_reset:
            raise RuntimeError('Tried to reset an environment before done. If you want to '
                               'allow early resets, wrap your env with Monitor(env, path, '
                               'allow_early_resets=True)')
        self.rewards = []
        self.needs_reset = False
        for key in self.reset_keywords:
            if kwargs.get(key) is None:
                raise ValueError('Expected you to pass kwarg %s into reset' % key)
            self.current_reset_info[key] = kwargs[key]
        return self.env.reset(**kwargs)

    def step(self, action):
        if self.needs_reset:
            raise RuntimeError('Tried to step environment that needs reset')
        observation, reward, done, info = self.env.step(action)
        self.rewards.append(reward)
        if done:
            self.needs_reset = True
            elapsed = time.time() - self.t_start
            ep_info = {'r': round(sum(self.rewards), 6), 'l': len(self.rewards),
                       't': round(elapsed, 6)}
            for key in self.info_keywords:
                ep_info[key] = info[key]
            self.episode_rewards.append(sum(self.rewards))
            self.episode_lengths.append(len(self.rewards))
            self.episode_times.append(elapsed)
            ep_info.update(self.current_reset_info)
            self.data.append(ep_info)
            if len(self.data) >= self.chunk_size:
                self.save()
            info['episode'] = ep_info
        self.total_steps += 1
        return observation, reward, done, info

    def close(self):
        if self.data:
            self.save()
        return self.env.close()

    def get_total_steps(self):
        return self.total_steps

    def get_episode_rewards(self):
        return self.episode_rewards

    def get_episode_lengths(self):
        return self.episode_lengths

    def get_episode_times(self):
        return self.episode_times
