"""custom_envs.utils.utils_venv: the older VecEnv module (``if done:`` auto-reset,
utils_venv.py:31), the same classes as custom_envs.vectorize."""
from custom_envs_amd.vectorize.concurrent import ConcurrentVecEnv, SubprocVecEnv, ThreadVecEnv

__all__ = ['ConcurrentVecEnv', 'SubprocVecEnv', 'ThreadVecEnv']
