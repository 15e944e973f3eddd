"""custom_envs.data.load_data (custom_envs/data/load_data.py:47-112)."""
from custom_envs_amd.data import load_data
from custom_envs_amd.data.files import load_emnist, load_mnist

__all__ = ['load_data', 'load_emnist', 'load_mnist']
