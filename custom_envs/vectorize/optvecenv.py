"""custom_envs.vectorize.optvecenv: multi-agent rows on one engine."""
from custom_envs_amd.vectorize.optvecenv import OptEnvRunner, OptVecEnv, flatten_dictionary

__all__ = ['OptEnvRunner', 'OptVecEnv', 'flatten_dictionary']
