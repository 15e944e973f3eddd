"""custom_envs_amd: MI355X-native engine for the custom_envs Optimize envs.

Registry ids and ``make`` keywords follow custom_envs/__init__.py:12-40.
Importing the package never touches the GPU; constructing an engine-backed
env loads the in-tree HIP library (custom_envs_amd/lib) and raises
``NativeEngineError`` if it is missing -- there is no CPU fallback.
"""
from custom_envs_amd.core import Env, Wrapper, make, register, registry
from custom_envs_amd.data import load_data
from custom_envs_amd._native import NativeEngineError

register(id='Optimize-v0', entry_point='custom_envs_amd.envs.optimize:Optimize')
register(id='MultiOptLRs-v0', entry_point='custom_envs_amd.envs.multioptlrs:MultiOptLRs')
register(id='MultiOptimize-v0',
         entry_point='custom_envs_amd.envs.multioptimize:MultiOptimize')

__all__ = ['Env', 'Wrapper', 'make', 'register', 'registry', 'load_data',
           'NativeEngineError']
