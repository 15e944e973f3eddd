"""Environments: the engine-backed Optimize-v0 / MultiOptLRs-v0 and the
host-side base classes (custom_envs/envs/__init__.py:1-9)."""
from custom_envs_amd.envs.baseenvironment import BaseEnvironment, BaseMultiEnvironment
from custom_envs_amd.envs.multioptimize import MultiOptimize
from custom_envs_amd.envs.multioptlrs import MultiOptLRs
from custom_envs_amd.envs.optimize import Optimize

SINGLE_AGENT_ENVIRONMENTS = (MultiOptimize, MultiOptLRs)

__all__ = ['BaseEnvironment', 'BaseMultiEnvironment', 'MultiOptimize', 'MultiOptLRs',
           'Optimize', 'SINGLE_AGENT_ENVIRONMENTS']
