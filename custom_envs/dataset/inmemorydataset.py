"""custom_envs.dataset.inmemorydataset."""
from custom_envs_amd.dataset import InMemoryDataSet

__all__ = ['InMemoryDataSet']
