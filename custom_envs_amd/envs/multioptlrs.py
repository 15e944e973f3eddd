"""MultiOptLRs-v0: one agent per problem parameter picks a log learning rate.

Reference: custom_envs/envs/multioptlrs.py:19-138 (version (3, 3, 0, 6)).
A single env is a one-env view of the HIP engine with auto-reset off; the
vector path is ``custom_envs_amd.vectorize.OptVecEnv``.  Same constructor
keywords (``problem``, ``max_batches``, ``max_history``), same Dict spaces
keyed 'parameter-i', same 14 info keys.  ``problem`` is 'func' (the
reference default: 2-D Rosenbrock from [-1.9, 2.0]), 'func4' (the configs'
4-D sum of two Rosenbrocks; ``initial_points`` overrides the start) or 'nn'
(get_problem('nn'): the OptimizeNN network, one agent per parameter;
``data_set`` is an InMemoryDataSet -- default the iris-shaped stand-in of
load_data() -- and ``hidden`` the create_neural_net layers, default
(256, 256)).
"""
import os

import numpy as np

from custom_envs_amd import _native
from custom_envs_amd.core import Env
from custom_envs_amd.multi_engine import agent_names, create_engine
from custom_envs_amd.spaces import Box, Dict


def multi_spaces(n_params, max_history):
    """utils_env.py:9-47 (v3) and :50-68 (v2), one Box per agent."""
    names = agent_names(n_params)
    obs = Box(low=-1e6, high=1e6, dtype=np.float32, shape=(3 * max_history,))
    act = Box(low=-1e3, high=1e4, dtype=np.float32, shape=(1,))
    return Dict({n: obs for n in names}), Dict({n: act for n in names})


def info_dict(row, terminal, reward, length):
    info = {k: float(v) for k, v in zip(_native.MULTI_INFO_KEYS, row)}
    info['loss'] = info['loss'] if terminal else None
    info['episode'] = {'r': reward, 'l': length}
    return info


class MultiOptLRs(Env):
    AGENT_FMT = 'parameter-{:d}'

    def __init__(self, problem='func', max_batches=400, max_history=5, initial_points=None,
                 device=0, data_set=None, hidden=None):
        self.spec_kwargs = {'problem': problem, 'max_batches': max_batches,
                            'max_history': max_history, 'initial_points': initial_points}
        if problem == 'nn':
            self.spec_kwargs.update(data_set=data_set, hidden=hidden)
        self.engine = create_engine(1, device=device, auto_reset=False, **self.spec_kwargs)
        ndims = self.engine.n_params
        self.max_batches, self.max_history = max_batches, max_history
        self.names = agent_names(ndims)
        self.observation_space, self.action_space = multi_spaces(ndims, max_history)
        self.current_step = 0
        self._rows = self.engine.row_agents

    def __repr__(self):
        return '<MultiOptLRs(VersionType(history=3, observation=3, action=0, reward=6))>'

    def _states(self, obs):
        return {self.names[agent]: obs[r].copy() for r, agent in enumerate(self._rows)}

    def seed(self, seed=None):
        """BaseEnvironment.seed (baseenvironment.py:20-28): None draws a seed
        from os.urandom, as gym's np_random does.  Only the 'nn' problem
        draws anything (its initial weights and shuffles)."""
        if seed is None:
            seed = int.from_bytes(os.urandom(8), 'little')
        self.engine.seed([seed])
        return [seed]

    def reset(self):
        self.current_step = 0
        return self._states(self.engine.reset())

    def step(self, action):
        rows = np.array([np.asarray(action[self.names[agent]], np.float32).ravel()[0]
                         for agent in self._rows], np.float32)
        out = self.engine.step(rows)
        self.current_step = int(out['episode_len'][0])
        terminal = bool(out['done'][0])
        reward = float(out['reward'][0])
        info = info_dict(out['info'][0], terminal, reward, self.current_step)
        return self._states(out['obs']), reward, terminal, info

    def close(self):
        self.engine.close()
