"""custom_envs.vectorize.concurrentvecenv: same-spec factories batch into one engine."""
from custom_envs_amd.vectorize.concurrent import ConcurrentVecEnv, SubprocVecEnv, ThreadVecEnv

__all__ = ['ConcurrentVecEnv', 'SubprocVecEnv', 'ThreadVecEnv']
