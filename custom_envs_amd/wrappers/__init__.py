"""Env wrappers (custom_envs/wrappers): host-side, unchanged semantics."""
from custom_envs_amd.wrappers.optimizewrappers import HistoryWrapper, SubSetWrapper
from custom_envs_amd.wrappers.monitor import Monitor

__all__ = ['HistoryWrapper', 'SubSetWrapper', 'Monitor']
