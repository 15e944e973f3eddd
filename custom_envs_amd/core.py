"""gym-style ``Env`` / ``Wrapper`` and the env-id registry.

The reference registers its envs with ``gym.envs.registration.register``
(custom_envs/__init__.py:12-40) and is driven through ``gym.make(id,
**kwargs)``.  gym is absent here, so the package keeps its own registry with
the same ids and kwargs; when gym *is* importable the ids are also
registered with gym so ``gym.make('Optimize-v0', ...)`` keeps working.
"""
import importlib


class Env:
    """Old-gym Env: 4-tuple step, reset -> obs, seed -> list."""
    metadata = {'render.modes': []}
    reward_range = (-float('inf'), float('inf'))
    spec = None
    observation_space = None
    action_space = None

    def step(self, action):
        raise NotImplementedError

    def reset(self):
        raise NotImplementedError

    def render(self, mode='human'):
        pass

    def close(self):
        pass

    def seed(self, seed=None):
        return [seed]

    @property
    def unwrapped(self):
        return self

    def __enter__(self):
        return self

    def __exit__(self, *args):
        self.close()
        return False


class Wrapper(Env):
    """gym.core.Wrapper: forwards everything it does not override."""

    def __init__(self, env):
        self.env = env
        self._observation_space = None
        self._action_space = None

    def __getattr__(self, name):
        if name.startswith('_'):
            raise AttributeError(name)
        return getattr(self.env, name)

    @property
    def observation_space(self):
        return self.env.observation_space if self._observation_space is None \
            else self._observation_space

    @observation_space.setter
    def observation_space(self, space):
        self._observation_space = space

    @property
    def action_space(self):
        return self.env.action_space if self._action_space is None else self._action_space

    @action_space.setter
    def action_space(self, space):
        self._action_space = space

    def step(self, action):
        return self.env.step(action)

    def reset(self, **kwargs):
        return self.env.reset(**kwargs)

    def render(self, mode='human', **kwargs):
        return self.env.render(mode, **kwargs)

    def close(self):
        return self.env.close()

    def seed(self, seed=None):
        return self.env.seed(seed)

    @property
    def unwrapped(self):
        return self.env.unwrapped


class EnvSpec:
    def __init__(self, env_id, entry_point, kwargs=None):
        self.id = env_id
        self.entry_point = entry_point
        self.kwargs = dict(kwargs or {})

    def load(self):
        module, attr = self.entry_point.split(':')
        return getattr(importlib.import_module(module), attr)

    def make(self, **kwargs):
        merged = dict(self.kwargs)
        merged.update(kwargs)
        env = self.load()(**merged)
        env.spec = self
        return env


registry = {}


def register(id, entry_point, **kwargs):  # noqa: A002 (gym's keyword name)
    registry[id] = EnvSpec(id, entry_point, kwargs.get('kwargs'))
    try:  # keep gym.make working where gym exists
        from gym.envs.registration import register as gym_register
        from gym.envs.registration import registry as gym_registry
        if id not in getattr(gym_registry, 'env_specs', {}):
            gym_register(id=id, entry_point=entry_point)
    except Exception:  # gym absent or incompatible: own registry only
        pass


def make(id, **kwargs):  # noqa: A002
    if id not in registry:
        raise KeyError('unknown environment id %r' % id)
    return registry[id].make(**kwargs)


def is_make(func):
    """True for this package's ``make`` and for ``gym.make``: the agent
    scripts build env factories as ``partial(gym.make, id, **kw)``
    (search_optimize_hyperparam.py:100-103, play_optimize.py:106-107), and
    with gym present the ids registered above resolve to this package."""
    if func is make:
        return True
    module = getattr(func, '__module__', None) or ''
    return getattr(func, '__name__', None) == 'make' and module.split('.')[0] == 'gym'


def make_request(fn):
    """(env id, kwargs) a factory ``partial(make | gym.make, id, **kw)``
    stands for, or None."""
    import functools
    if (isinstance(fn, functools.partial) and is_make(fn.func) and len(fn.args) == 1
            and fn.args[0] in registry):
        return fn.args[0], dict(fn.keywords)
    return None
