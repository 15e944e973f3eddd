"""custom_envs.envs.multioptlrs: MultiOptLRs-v0 on the HIP engine."""
from custom_envs_amd.envs.multioptlrs import MultiOptLRs

__all__ = ['MultiOptLRs']
