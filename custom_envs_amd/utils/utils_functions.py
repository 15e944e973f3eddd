"""Test functions for the function problems (utils_functions.py:4-6)."""


def compute_rosenbrock(x, y):
    """Rosenbrock 100 (y - x^2)^2 + (1 - x)^2 (utils_functions.py:4-6); the
    engine's 'func'/'func4' problems evaluate it in-kernel in float32."""
    return 100 * (y - x ** 2) ** 2 + (1 - x) ** 2
