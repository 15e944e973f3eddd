"""custom_envs.envs.baseenvironment."""
from custom_envs_amd.envs.baseenvironment import BaseEnvironment, BaseMultiEnvironment

__all__ = ['BaseEnvironment', 'BaseMultiEnvironment']
