"""custom_envs.envs (custom_envs/envs/__init__.py:1-9)."""
from custom_envs_amd.envs import (SINGLE_AGENT_ENVIRONMENTS, BaseEnvironment,
                                  BaseMultiEnvironment, MultiOptimize, MultiOptLRs, Optimize)

__all__ = ['BaseEnvironment', 'BaseMultiEnvironment', 'MultiOptimize', 'MultiOptLRs',
           'Optimize', 'SINGLE_AGENT_ENVIRONMENTS']
