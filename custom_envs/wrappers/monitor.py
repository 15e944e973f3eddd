"""custom_envs.wrappers.monitor (the stable-baselines-style Monitor)."""
from custom_envs_amd.wrappers.monitor import Monitor

__all__ = ['Monitor']
