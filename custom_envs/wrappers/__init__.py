"""custom_envs.wrappers."""
from custom_envs_amd.wrappers import HistoryWrapper, Monitor, SubSetWrapper

__all__ = ['HistoryWrapper', 'Monitor', 'SubSetWrapper']
