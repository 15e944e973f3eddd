"""Restatement of ``custom_envs.vectorize`` (TEST/BASELINE INFRASTRUCTURE ONLY).

``custom_envs/vectorize/concurrentvecenv.py:16-271``: one worker (thread or
process) and one duplex ``multiprocessing.Pipe`` per env, a pickled
``(cmd, data)`` loop in the worker, ``np.stack`` of the per-env results in
``step_wait``.  Auto-reset uses the working single-agent form ``if done:``
of ``custom_envs/utils/utils_venv.py:31`` (``any(done)`` at
``concurrentvecenv.py:37`` raises on a bool); ``np.any`` covers both the
bool of a single env and the per-agent lists of ``OptEnvRunner``.

This is the CPU baseline ``bench.py`` times beside the GPU engine: the
reference's own NumPy vectorisation path, restated because the reference
itself cannot import here (gym, stable_baselines and ModelNumpy missing).
"""
import multiprocessing as mp
import pickle
from threading import Thread

import numpy as np


class _Payload:
    """cloudpickle wrapper for env factories (SB ``CloudpickleWrapper``)."""

    def __init__(self, fn):
        self.fn = fn

    def __getstate__(self):
        import cloudpickle
        return cloudpickle.dumps(self.fn)

    def __setstate__(self, blob):
        self.fn = pickle.loads(blob)


def _worker(remote, payload):
    env = payload.fn()
    try:
        while True:
            cmd, data = remote.recv()
            if cmd == 'step':
                obs, reward, done, info = env.step(data)
                if np.any(done):
                    obs = env.reset()
                remote.send((obs, reward, done, info))
            elif cmd == 'reset':
                remote.send(env.reset())
            elif cmd == 'close':
                remote.close()
                break
            elif cmd == 'get_spaces':
                remote.send((getattr(env, 'observation_space', None),
                             getattr(env, 'action_space', None)))
            elif cmd == 'env_method':
                remote.send(getattr(env, data[0])(*data[1], **data[2]))
            elif cmd == 'get_attr':
                remote.send(getattr(env, data))
            elif cmd == 'set_attr':
                remote.send(setattr(env, data[0], data[1]))
            else:
                raise NotImplementedError(cmd)
    except EOFError:
        pass
    finally:
        env.close()


class ConcurrentVecEnv:
    """concurrentvecenv.py:67-200."""

    def __init__(self, env_fns, create_method):
        self.waiting = False
        self.closed = False
        pipes = [mp.Pipe(True) for _ in env_fns]
        self.remotes = [p[0] for p in pipes]
        self.work_remotes = [p[1] for p in pipes]
        self.processes = []
        for work_remote, env_fn in zip(self.work_remotes, env_fns):
            proc = create_method(target=_worker,
                                 args=(work_remote, _Payload(env_fn)),
                                 daemon=True)
            proc.start()
            self.processes.append(proc)
        self.num_envs = len(env_fns)
        self.remotes[0].send(('get_spaces', None))
        self.observation_space, self.action_space = self.remotes[0].recv()

    def step_async(self, actions):
        for remote, action in zip(self.remotes, actions):
            remote.send(('step', action))
        self.waiting = True

    def step_wait(self):
        results = [remote.recv() for remote in self.remotes]
        self.waiting = False
        obs, rews, dones, infos = zip(*results)
        return np.stack(obs), np.stack(rews), np.stack(dones), infos

    def step(self, actions):
        self.step_async(actions)
        return self.step_wait()

    def reset(self):
        for remote in self.remotes:
            remote.send(('reset', None))
        return np.stack([remote.recv() for remote in self.remotes])

    def env_method(self, name, *args, **kwargs):
        for remote in self.remotes:
            remote.send(('env_method', (name, args, kwargs)))
        return [remote.recv() for remote in self.remotes]

    def get_attr(self, name):
        for remote in self.remotes:
            remote.send(('get_attr', name))
        return [remote.recv() for remote in self.remotes]

    def close(self):
        if self.closed:
            return
        if self.waiting:
            for remote in self.remotes:
                remote.recv()
        for remote in self.remotes:
            remote.send(('close', None))
        for proc in self.processes:
            proc.join()
        self.closed = True


class ThreadVecEnv(ConcurrentVecEnv):
    """concurrentvecenv.py:254-271."""

    def __init__(self, env_fns):
        super().__init__(env_fns, Thread)


class SubprocVecEnv(ConcurrentVecEnv):
    """concurrentvecenv.py:233-251 (start method fork/forkserver/spawn)."""

    def __init__(self, env_fns, start_method=None):
        if start_method is None:
            start_method = ('forkserver' if 'forkserver'
                            in mp.get_all_start_methods() else 'spawn')
        super().__init__(env_fns, mp.get_context(start_method).Process)
