"""custom_envs.wrappers.optimizewrappers."""
from custom_envs_amd.wrappers.optimizewrappers import HistoryWrapper, SubSetWrapper

__all__ = ['HistoryWrapper', 'SubSetWrapper']
