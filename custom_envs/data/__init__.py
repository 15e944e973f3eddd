"""custom_envs.data."""
from custom_envs_amd.data import load_data

__all__ = ['load_data']
