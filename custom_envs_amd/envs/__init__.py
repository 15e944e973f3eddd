"""Environments backed by the HIP engine."""
from custom_envs_amd.envs.optimize import Optimize

__all__ = ['Optimize']
