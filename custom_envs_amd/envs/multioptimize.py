"""MultiOptimize-v0 (custom_envs/envs/multioptimize.py), kept importable.

The reference's constructor cannot succeed: it calls
``get_problem(data_set=load_data(...))`` (multioptimize.py:44), which hands
``data_set`` to ``OptimizeFunction.create`` (problems/__init__.py:7-16), a
keyword that method does not take -> TypeError.  The class stays importable
because run_multiagent_exp_single.py:24 imports it, and constructing it
fails the way the reference does.  SURVEY.md 2, row 4: out of scope.
"""
from custom_envs_amd.envs.baseenvironment import BaseMultiEnvironment


class MultiOptimize(BaseMultiEnvironment):
    def __init__(self, data_set='iris', batch_size=None, version=1, max_batches=400,
                 max_history=5, observation_version=0, action_version=0, reward_version=0):
        raise TypeError("create() got an unexpected keyword argument 'data_set' "
                        "(MultiOptimize: get_problem(data_set=...) at multioptimize.py:44 "
                        "reaches OptimizeFunction.create, as in the reference)")
