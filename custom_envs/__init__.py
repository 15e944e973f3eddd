"""Drop-in import surface of the reference package ``custom_envs``.

Every module path the reference's callers import resolves here to the
MI355X engine package ``custom_envs_amd`` (custom_envs/__init__.py:1-40 and
the modules below): the agent scripts keep their import lines
(play_optimize.py:21-25, run_multiagent_exp_single.py:21-25,
search_optimize_hyperparam.py:15-16, eval_exp.py:15).  Importing registers
the env ids with this package's registry and, when gym is importable, with
gym, so ``gym.make('Optimize-v0', ...)`` builds the engine-backed env.
"""
from custom_envs_amd import NativeEngineError, make, register, registry
from custom_envs_amd.data import load_data

__all__ = ['NativeEngineError', 'load_data', 'make', 'register', 'registry']
