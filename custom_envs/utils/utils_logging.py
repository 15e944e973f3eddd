"""custom_envs.utils.utils_logging (Monitor, create_env; VecMonitor batches them)."""
from custom_envs_amd.utils.utils_logging import Monitor, VecMonitor, create_env

__all__ = ['Monitor', 'VecMonitor', 'create_env']
