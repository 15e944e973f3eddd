"""custom_envs.utils.utils_math."""
from custom_envs_amd.utils.utils_math import (cross_entropy, mse, normalize, sigmoid, softmax,
                                              use_random_state)

__all__ = ['cross_entropy', 'mse', 'normalize', 'sigmoid', 'softmax', 'use_random_state']
