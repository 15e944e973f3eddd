"""custom_envs.utils.utils_common (History, shuffle, to_onehot, flat arrays)."""
from custom_envs_amd.utils.utils_common import (History, flatten_arrays, from_flat, shuffle,
                                                to_onehot)

__all__ = ['History', 'flatten_arrays', 'from_flat', 'shuffle', 'to_onehot']
