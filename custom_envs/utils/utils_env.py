"""custom_envs.utils.utils_env."""
from custom_envs_amd.utils.utils_env import (get_action_optlrs, get_action_space_optlrs,
                                             get_obs_version, get_observation, get_reward)

__all__ = ['get_action_optlrs', 'get_action_space_optlrs', 'get_obs_version',
           'get_observation', 'get_reward']
