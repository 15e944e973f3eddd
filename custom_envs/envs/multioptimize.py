"""custom_envs.envs.multioptimize (importable; its constructor fails as the reference's)."""
from custom_envs_amd.envs.multioptimize import MultiOptimize

__all__ = ['MultiOptimize']
