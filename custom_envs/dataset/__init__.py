"""custom_envs.dataset."""
from custom_envs_amd.dataset import BatchType, DataSet, InMemoryDataSet

__all__ = ['BatchType', 'DataSet', 'InMemoryDataSet']
