"""``ThreadVecEnv`` / ``SubprocVecEnv``: the reference's constructor surface.

custom_envs/vectorize/concurrentvecenv.py:233-271 takes a list of env
factories and runs each env in its own thread/process behind a pipe.  Here
the same constructors first look at the factories: when every one builds the
same registered engine-backed id with the same keywords (e.g.
``[partial(make, 'Optimize-v0', data_set=...)] * n``), the whole batch
becomes ONE ``GPUVecEnv`` -- one fused kernel per step instead of n worker
round trips.  Any other factory list (stub envs, third-party envs) runs on
the generic host workers below, with the reference's command set and the
``if done: reset`` auto-reset of custom_envs/utils/utils_venv.py:31.
"""
import functools
import multiprocessing as mp
import pickle
import threading

import numpy as np

from custom_envs_amd.spaces import Dict

ENGINE_IDS = {'Optimize-v0'}


def _engine_request(env_fns):
    """(env_id, kwargs) if all factories build the same engine-backed env."""
    from custom_envs_amd.core import make
    from custom_envs_amd.envs.optimize import Optimize
    first = None
    for fn in env_fns:
        if not isinstance(fn, functools.partial):
            return None
        if fn.func is make and len(fn.args) == 1 and fn.args[0] in ENGINE_IDS:
            req = (fn.args[0], dict(fn.keywords))
        elif fn.func is Optimize and not fn.args:
            req = ('Optimize-v0', dict(fn.keywords))
        else:
            return None
        if first is None:
            first = req
        elif req != first:
            return None
    return first


class _Cloud:
    """Ship a factory to a worker with cloudpickle (closures, lambdas)."""

    def __init__(self, fn):
        self.fn = fn

    def __getstate__(self):
        import cloudpickle
        return cloudpickle.dumps(self.fn)

    def __setstate__(self, blob):
        self.fn = pickle.loads(blob)


def _serve(conn, factory):
    env = factory.fn()

    def do_step(action):
        obs, reward, done, info = env.step(action)
        if np.any(done):
            obs = env.reset()
        return obs, reward, done, info

    handlers = {
        'step': do_step,
        'reset': lambda _: env.reset(),
        'render': lambda data: env.render(*data[0], **data[1]),
        'get_spaces': lambda _: (env.observation_space, env.action_space),
        'env_method': lambda data: getattr(env, data[0])(*data[1], **data[2]),
        'get_attr': lambda name: getattr(env, name),
        'set_attr': lambda data: setattr(env, data[0], data[1]),
    }
    try:
        while True:
            cmd, data = conn.recv()
            if cmd == 'close':
                conn.close()
                return
            conn.send(handlers[cmd](data))
    except EOFError:
        pass
    finally:
        env.close()


def stack_obs(obs, space):
    if isinstance(space, Dict) or (obs and isinstance(obs[0], dict)):
        keys = space.spaces.keys() if isinstance(space, Dict) else obs[0].keys()
        return {k: np.stack([o[k] for o in obs]) for k in keys}
    if obs and isinstance(obs[0], tuple):
        return tuple(np.stack(col) for col in zip(*obs))
    return np.stack(obs)


class ConcurrentVecEnv:
    """One worker per env, or one GPU engine when the factories allow it."""

    def __init__(self, env_fns, spawn):
        self.closed = False
        self.waiting = False
        request = _engine_request(env_fns)
        self._gpu = None
        if request is not None:
            from custom_envs_amd.vectorize.gpuvecenv import GPUVecEnv
            self._gpu = GPUVecEnv(len(env_fns), **request[1])
            self.num_envs = self._gpu.num_envs
            self.observation_space = self._gpu.observation_space
            self.action_space = self._gpu.action_space
            return
        self.remotes, self.processes = [], []
        for fn in env_fns:
            parent, child = mp.Pipe(duplex=True)
            worker = spawn(target=_serve, args=(child, _Cloud(fn)), daemon=True)
            worker.start()
            self.remotes.append(parent)
            self.processes.append(worker)
        self.num_envs = len(env_fns)
        self.observation_space, self.action_space = self._call_one(0, 'get_spaces', None)

    @property
    def engine_backed(self):
        return self._gpu is not None

    def _call_one(self, i, cmd, data):
        self.remotes[i].send((cmd, data))
        return self.remotes[i].recv()

    def _broadcast(self, cmd, data, indices=None):
        targets = range(self.num_envs) if indices is None else (
            [indices] if isinstance(indices, int) else indices)
        remotes = [self.remotes[i] for i in targets]
        for remote in remotes:
            remote.send((cmd, data))
        return [remote.recv() for remote in remotes]

    def step_async(self, actions):
        if self._gpu is not None:
            self._gpu.step_async(actions)
        else:
            for remote, action in zip(self.remotes, actions):
                remote.send(('step', action))
        self.waiting = True

    def step_wait(self):
        self.waiting = False
        if self._gpu is not None:
            return self._gpu.step_wait()
        obs, rews, dones, infos = zip(*[remote.recv() for remote in self.remotes])
        return stack_obs(obs, self.observation_space), np.stack(rews), np.stack(dones), infos

    def step(self, actions):
        self.step_async(actions)
        return self.step_wait()

    def reset(self):
        if self._gpu is not None:
            return self._gpu.reset()
        return stack_obs(self._broadcast('reset', None), self.observation_space)

    def seed(self, seed=None):
        if self._gpu is not None:
            return self._gpu.seed(seed)
        seeds = [None if seed is None else seed + i for i in range(self.num_envs)]
        return [self._call_one(i, 'env_method', ('seed', (s,), {})) for i, s in enumerate(seeds)]

    def render(self, *args, **kwargs):
        if self._gpu is not None:
            return None
        return self._broadcast('render', (args, kwargs))

    def get_images(self):
        if self._gpu is not None:
            return self._gpu.get_images()
        return self._broadcast('render', ((), {'mode': 'rgb_array'}))

    def env_method(self, method_name, *method_args, indices=None, **method_kwargs):
        if self._gpu is not None:
            return self._gpu.env_method(method_name, *method_args, indices=indices,
                                        **method_kwargs)
        return self._broadcast('env_method', (method_name, method_args, method_kwargs), indices)

    def get_attr(self, attr_name, indices=None):
        if self._gpu is not None:
            return self._gpu.get_attr(attr_name, indices)
        return self._broadcast('get_attr', attr_name, indices)

    def set_attr(self, attr_name, value, indices=None):
        if self._gpu is not None:
            return self._gpu.set_attr(attr_name, value, indices)
        return self._broadcast('set_attr', (attr_name, value), indices)

    def close(self):
        if self.closed:
            return
        self.closed = True
        if self._gpu is not None:
            self._gpu.close()
            return
        if self.waiting:
            for remote in self.remotes:
                remote.recv()
        for remote in self.remotes:
            remote.send(('close', None))
        for proc in self.processes:
            proc.join()


class ThreadVecEnv(ConcurrentVecEnv):
    def __init__(self, env_fns):
        super().__init__(env_fns, threading.Thread)


class SubprocVecEnv(ConcurrentVecEnv):
    def __init__(self, env_fns, start_method=None):
        if start_method is None:
            start_method = 'forkserver' if 'forkserver' in mp.get_all_start_methods() else 'spawn'
        super().__init__(env_fns, mp.get_context(start_method).Process)
