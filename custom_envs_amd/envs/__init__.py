"""Environments backed by the HIP engine."""
from custom_envs_amd.envs.multioptlrs import MultiOptLRs
from custom_envs_amd.envs.optimize import Optimize

__all__ = ['MultiOptLRs', 'Optimize']
