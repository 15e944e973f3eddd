"""Stable-baselines ``VecEnv`` over one HIP engine: E envs, one launch per step.

Replaces custom_envs/vectorize/concurrentvecenv.py:67-200 for Optimize-v0:
instead of one thread + one pickling pipe per env, ``step_async`` hands
the (E, P) action block to the engine (one H2D copy, one fused kernel, one
D2H copy of the packed outputs) and ``step_wait`` returns

  obs   (E, 2P+1) float32     np.stack of per-env observations
  rews  (E,)      float32     -loss per env
  dones (E,)      bool        current_step >= 40, envs auto-reset in-kernel
  infos           LazyInfos   sequence of {'objective', 'accuracy',
                              'episode': {'r', 'l'}} built on access

Auto-reset follows utils_venv.py:31 (``if done: obs = env.reset()``): the
returned obs of a finished env is its reset observation.
"""
import numpy as np

from custom_envs_amd.envs.optimize import optimize_spaces, resolve_dataset


class LazyInfos:
    """Per-env info dicts materialised on access (no O(E) dict build per step).

    ``episodes`` maps env index -> the Monitor's episode record for envs a
    ``VecMonitor`` closed this step (utils_logging.py:98-116 replaces
    ``info['episode']`` with it)."""

    def __init__(self, objective, accuracy, reward, episode_len, episodes=None):
        self._objective = objective
        self._accuracy = accuracy
        self._reward = reward
        self._episode_len = episode_len
        self.episodes = {} if episodes is None else episodes

    def __len__(self):
        return len(self._objective)

    def __getitem__(self, idx):
        if isinstance(idx, slice):
            return [self[i] for i in range(*idx.indices(len(self)))]
        if idx < 0:
            idx += len(self)
        reward = float(self._reward[idx])
        episode = self.episodes.get(idx)
        return {'objective': float(self._objective[idx]),
                'accuracy': float(self._accuracy[idx]),
                'episode': {'r': reward, 'l': int(self._episode_len[idx])}
                if episode is None else episode}

    def __iter__(self):
        return (self[i] for i in range(len(self)))

    def __repr__(self):
        return 'LazyInfos(n=%d)' % len(self)


class GPUVecEnv:
    """E Optimize-v0 envs on one MI355X behind the SB VecEnv interface."""

    def __init__(self, num_envs, data_set='gaussians_256x10', batch_size=None,
                 n_of_steps=None, max_steps=40, precision=None, device=0, seed=None,
                 model='linear', hidden=64, monitor=None, data_dir=None):
        """``monitor``: None, or (file paths, Monitor keywords) -- the batched
        form of wrapping every env in utils_logging.Monitor
        (utils_logging.py:159-175); writes the same ``.mon.csv`` chunks."""
        from custom_envs_amd.engine import OptimizeEngine
        from custom_envs_amd.utils.utils_logging import VecMonitor
        features, targets = resolve_dataset(data_set, batch_size, data_dir)
        self.engine = OptimizeEngine(features, targets, num_envs, batch_size=batch_size,
                                     max_steps=max_steps, precision=precision, device=device,
                                     auto_reset=True, model=model, hidden=hidden)
        self.num_envs = int(num_envs)
        self.observation_space, self.action_space = optimize_spaces(self.engine.act_dim)
        self.monitor = None
        if monitor is not None:
            paths, mkw = monitor
            self.monitor = VecMonitor(self.num_envs, paths,
                                      info_keywords=mkw.get('info_keywords', ()),
                                      chunk_size=mkw.get('chunk_size', 1),
                                      callbacks=mkw.get('callbacks'),
                                      style=mkw.get('style', 'logging'),
                                      allow_early_resets=mkw.get('allow_early_resets', True),
                                      reset_keywords=mkw.get('reset_keywords', ()))
        self.current_step = np.zeros(self.num_envs, np.int64)
        self.waiting = False
        self.closed = False
        self.seed(seed)

    # ----------------------------------------------------------- VecEnv API
    def seed(self, seed=None):
        """int -> env i gets seed + i; sequence -> per-env seeds; None -> random."""
        if seed is None or isinstance(seed, (int, np.integer)):
            return self.engine.seed(seed)
        return self.engine.seed(list(seed))

    @property
    def single_observation_space(self):
        """gym.vector.VectorEnv name of one env's space (SB's observation_space)."""
        return self.observation_space

    @property
    def single_action_space(self):
        return self.action_space

    def reset(self):
        self.current_step[:] = 0
        if self.monitor is not None:
            self.monitor.reset()
        return self.engine.reset()

    def step_async(self, actions):
        if self.monitor is not None:
            self.monitor.check_step()
        self.engine.step_async(actions)
        self.waiting = True

    def step_wait(self):
        out = self.engine.step_wait()
        self.waiting = False
        dones = out['done'].astype(bool)
        ep_len = out['episode_len'].copy()
        self.current_step[:] = np.where(dones, 0, ep_len)
        reward = out['reward'].copy()
        infos = LazyInfos(out['objective'].copy(), out['accuracy'].copy(), reward, ep_len)
        obs = out['obs'].copy()
        if self.monitor is not None:
            infos.episodes.update(self.monitor.step(reward, dones, infos, obs))
        return obs, reward, dones, infos

    def step(self, actions):
        self.step_async(actions)
        return self.step_wait()

    def close(self):
        if not self.closed:
            if self.monitor is not None:
                self.monitor.close()
            self.engine.close()
            self.closed = True

    def render(self, *args, **kwargs):
        return None

    def get_images(self):
        return [None] * self.num_envs

    def _indices(self, indices):
        if indices is None:
            return range(self.num_envs)
        if isinstance(indices, int):
            return [indices]
        return indices

    def get_attr(self, attr_name, indices=None):
        idx = self._indices(indices)
        if attr_name == 'current_step':
            return [int(self.current_step[i]) for i in idx]
        if attr_name in ('observation_space', 'action_space'):
            return [getattr(self, attr_name)] * len(idx)
        if attr_name == 'seeds':
            return [self.engine.seeds[i] for i in idx]
        state_keys = {'weights': 'weights', 'grad_hist': 'grad_hist', 'loss_hist': 'loss_hist'}
        if attr_name in state_keys:
            state = self.engine.get_state()[state_keys[attr_name]]
            return [state[i] for i in idx]
        raise AttributeError('GPUVecEnv has no per-env attribute %r' % attr_name)

    def set_attr(self, attr_name, value, indices=None):
        raise AttributeError('engine-backed envs have no settable attribute %r' % attr_name)

    def env_method(self, method_name, *method_args, indices=None, **method_kwargs):
        idx = list(self._indices(indices))
        if method_name == 'seed':
            seeds = list(self.engine.seeds)
            seed = method_args[0] if method_args else method_kwargs.get('seed')
            for i in idx:
                seeds[i] = seed
            self.engine.seed(seeds)
            return [[seeds[i]] for i in idx]
        if method_name in ('render', 'close'):
            return [None] * len(idx)
        monitor_methods = ('get_episode_rewards', 'get_episode_lengths', 'get_episode_times',
                           'get_total_steps')
        if method_name in monitor_methods and self.monitor is not None:
            return getattr(self.monitor, method_name)(idx)
        raise AttributeError('GPUVecEnv has no per-env method %r' % method_name)

    @property
    def unwrapped(self):
        return self

    def __len__(self):
        return self.num_envs

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def batch_space(space, n):
    """gym.vector.utils.batch_space for a Box: the stacked (n, ...) space."""
    from custom_envs_amd.spaces import Box
    return Box(low=np.broadcast_to(space.low, (n,) + space.shape),
               high=np.broadcast_to(space.high, (n,) + space.shape),
               shape=(n,) + space.shape, dtype=space.dtype)


class VectorEnv(GPUVecEnv):
    """The same engine behind the ``gym.vector.VectorEnv`` surface the north
    star names: ``observation_space``/``action_space`` are the batched
    spaces, ``single_observation_space``/``single_action_space`` one env's
    (GPUVecEnv keeps stable-baselines' convention, where the plain names are
    one env's spaces).  ``reset() -> obs``, ``step(actions) -> (obs, rewards,
    dones, infos)`` with auto-reset, as gym<=0.21's vector envs."""
    is_vector_env = True

    def __init__(self, num_envs, **kwargs):
        super().__init__(num_envs, **kwargs)
        self._single = (self.observation_space, self.action_space)
        self.observation_space = batch_space(self._single[0], self.num_envs)
        self.action_space = batch_space(self._single[1], self.num_envs)

    @property
    def single_observation_space(self):
        return self._single[0]

    @property
    def single_action_space(self):
        return self._single[1]

    def get_attr(self, attr_name, indices=None):
        if attr_name in ('observation_space', 'action_space'):
            space = self._single[0 if attr_name == 'observation_space' else 1]
            return [space] * len(self._indices(indices))
        return super().get_attr(attr_name, indices)


def make_vec(env_id, num_envs, **kwargs):
    """``gym.vector.make(id, num_envs, **kw)`` for the engine-backed ids: ONE
    engine for all envs instead of num_envs worker processes."""
    if env_id != 'Optimize-v0':
        raise KeyError('make_vec serves Optimize-v0; MultiOptLRs-v0 batches through OptVecEnv')
    return VectorEnv(num_envs, **kwargs)
