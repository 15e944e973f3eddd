"""custom_envs.vectorize (custom_envs/vectorize/__init__.py:1-3)."""
from custom_envs_amd.vectorize import (GPUVecEnv, OptVecEnv, SubprocVecEnv, ThreadVecEnv,
                                       VectorEnv, make_vec)

__all__ = ['GPUVecEnv', 'OptVecEnv', 'SubprocVecEnv', 'ThreadVecEnv', 'VectorEnv', 'make_vec']
