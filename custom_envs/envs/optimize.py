"""custom_envs.envs.optimize: Optimize-v0 on the HIP engine."""
from custom_envs_amd.envs.optimize import Optimize

__all__ = ['Optimize']
