"""custom_envs.utils.utils_functions."""
from custom_envs_amd.utils.utils_functions import compute_rosenbrock

__all__ = ['compute_rosenbrock']
