"""Vectorised environments (replaces custom_envs/vectorize/__init__.py:1-3)."""
from custom_envs_amd.vectorize.concurrent import SubprocVecEnv, ThreadVecEnv
from custom_envs_amd.vectorize.gpuvecenv import GPUVecEnv, LazyInfos, VectorEnv, make_vec
from custom_envs_amd.vectorize.optvecenv import OptEnvRunner, OptVecEnv

__all__ = ['GPUVecEnv', 'LazyInfos', 'OptEnvRunner', 'OptVecEnv', 'SubprocVecEnv',
           'ThreadVecEnv', 'VectorEnv', 'make_vec']
