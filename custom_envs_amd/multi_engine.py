"""Python handle on one HIP MultiOptLRs-v0 engine (E envs x P agents, one GPU).

Rows follow OptVecEnv's flattening (custom_envs/vectorize/optvecenv.py:
10-14): env-major, agents in sorted name order ('parameter-0',
'parameter-1', 'parameter-10', ...).  ``row_agents`` gives the agent index
of each row.  No CPU fallback: without the library or a GPU, construction
raises ``NativeEngineError``.
"""
import ctypes

import numpy as np

from custom_envs_amd import _native
from custom_envs_amd._native import CeMultiConfig, CeMultiOutputs, check

# problem names accepted by MultiOptLRs(problem=...): the reference's default
# 'func' (2-D Rosenbrock, start [-1.9, 2.0], optimize_function.py:35-37) and
# the configs' build-defined 4-D sum of two Rosenbrocks
PROBLEMS = {
    'func': (2, [-1.9, 2.0]),
    'func4': (4, [-1.9, 2.0, -1.9, 2.0]),
}


def agent_names(n_params):
    return ['parameter-{:d}'.format(i) for i in range(n_params)]


def row_agents(n_params):
    """Agent index of each OptVecEnv row (names sorted as strings)."""
    names = agent_names(n_params)
    return sorted(range(n_params), key=lambda i: names[i])


def resolve_problem(problem, initial_points=None):
    if isinstance(problem, str):
        if problem not in PROBLEMS:
            raise RuntimeError('Not a name of a problem: %r (the TF "nn" problem is out of '
                               'scope for the GPU engine)' % problem)
        ndims, start = PROBLEMS[problem]
    else:
        ndims = int(problem.get('ndims', 2))
        start = problem.get('initial_points')
    if initial_points is not None:
        start = list(initial_points)
    if start is None or len(start) != ndims:
        raise ValueError('initial_points must have ndims entries (the reference random '
                         'start is broken, optimize_function.py:34,43)')
    return ndims, [float(v) for v in start]


def _view(ptr, count, ctype, dtype, shape):
    return np.frombuffer((ctype * count).from_address(ptr), dtype=dtype).reshape(shape)


class MultiOptEngine:
    """E MultiOptLRs envs advanced in lock step; outputs in OptVecEnv rows."""

    def __init__(self, num_envs, problem='func', max_batches=400, max_history=5,
                 initial_points=None, device=0, auto_reset=True):
        lib = _native.load()
        ndims, start = resolve_problem(problem, initial_points)
        self.num_envs, self.n_params = int(num_envs), ndims
        self.max_history, self.max_batches = int(max_history), int(max_batches)
        cfg = CeMultiConfig(abi_version=_native.ABI_VERSION, device=int(device),
                            num_envs=self.num_envs, n_params=ndims,
                            function=_native.CE_FUNC_ROSENBROCK_PAIRS,
                            max_history=self.max_history, max_batches=self.max_batches,
                            auto_reset=1 if auto_reset else 0)
        for i, v in enumerate(start):
            cfg.initial_points[i] = v
        handle = ctypes.c_void_p()
        check(lib.ce_multi_create(ctypes.byref(cfg), ctypes.byref(handle)), 'ce_multi_create')
        self._lib, self._h = lib, handle
        self.row_agents = row_agents(ndims)
        view = CeMultiOutputs()
        check(lib.ce_multi_host_outputs(handle, ctypes.byref(view)), 'ce_multi_host_outputs')
        E, P, W = self.num_envs, ndims, 3 * self.max_history
        n_info = len(_native.MULTI_INFO_KEYS)
        self._host = {
            'obs': _view(view.obs, E * P * W, ctypes.c_float, np.float32, (E * P, W)),
            'reward': _view(view.reward, E * P, ctypes.c_float, np.float32, (E * P,)),
            'done': _view(view.done, E * P, ctypes.c_uint8, np.uint8, (E * P,)),
            'info': _view(view.info, E * n_info, ctypes.c_float, np.float32, (E, n_info)),
            'episode_len': _view(view.episode_len, E, ctypes.c_int32, np.int32, (E,)),
        }

    def seed(self, seeds=None):
        """MultiOptLRs draws nothing at reset (fixed initial_points): seeds are
        accepted for the VecEnv surface and ignored, like the reference's
        unused RNG (multioptlrs.py:39-48)."""
        return seeds

    @property
    def rows(self):
        return self.num_envs * self.n_params

    def reset(self):
        check(self._lib.ce_multi_reset(self._h, None, 0), 'ce_multi_reset')
        return self._host['obs'].copy()

    def step_async(self, actions):
        actions = np.ascontiguousarray(actions, dtype=np.float32).reshape(self.rows)
        self._pending = actions
        check(self._lib.ce_multi_step_async(self._h, actions.ctypes.data, None, 0),
              'ce_multi_step_async')

    def step_wait(self):
        check(self._lib.ce_multi_wait(self._h), 'ce_multi_wait')
        self._pending = None
        return self._host

    def step(self, actions):
        self.step_async(actions)
        return self.step_wait()

    # ------------------------------------------------------------- device mode
    def set_stream(self, stream_handle):
        check(self._lib.ce_multi_set_stream(self._h, ctypes.c_void_p(stream_handle or 0)),
              'ce_multi_set_stream')

    def output_fields(self):
        """(name, torch dtype, rows per env, trailing shape) of the step outputs."""
        import torch
        P, W = self.n_params, 3 * self.max_history
        return [('obs', torch.float32, P, (W,)),
                ('reward', torch.float32, P, ()),
                ('done', torch.uint8, P, ()),
                ('info', torch.float32, 1, (len(_native.MULTI_INFO_KEYS),)),
                ('episode_len', torch.int32, 1, ())]

    def alloc_device_outputs(self, torch_device=None):
        import torch
        dev = torch_device or torch.device('cuda')
        return {name: torch.empty((self.num_envs * rows,) + tail, dtype=dtype, device=dev)
                for name, dtype, rows, tail in self.output_fields()}

    @staticmethod
    def _outputs(out):
        return CeMultiOutputs(obs=out['obs'].data_ptr(), reward=out['reward'].data_ptr(),
                              done=out['done'].data_ptr(), info=out['info'].data_ptr(),
                              episode_len=out['episode_len'].data_ptr())

    def reset_device(self, out):
        o = self._outputs(out)
        check(self._lib.ce_multi_reset(self._h, ctypes.byref(o), _native.CE_PTR_DEVICE),
              'ce_multi_reset')

    def step_device(self, actions, out):
        if actions.numel() < self.rows or not actions.is_contiguous():
            raise ValueError('actions must be a contiguous float32 tensor of E*P rows')
        o = self._outputs(out)
        check(self._lib.ce_multi_step_async(self._h, actions.data_ptr(), ctypes.byref(o),
                                            _native.CE_PTR_DEVICE), 'ce_multi_step_async')

    def step_many_device(self, k, actions, out, per_step_actions=True):
        if actions.numel() < (k if per_step_actions else 1) * self.rows:
            raise ValueError('actions tensor too small')
        o = self._outputs(out)
        stride = self.rows if per_step_actions else 0
        check(self._lib.ce_multi_step_many(self._h, int(k), actions.data_ptr(), stride,
                                           ctypes.byref(o)), 'ce_multi_step_many')

    def wait(self):
        check(self._lib.ce_multi_wait(self._h), 'ce_multi_wait')

    def get_state(self):
        theta = np.zeros((self.num_envs, self.n_params), np.float32)
        step = np.zeros(self.num_envs, np.int32)
        check(self._lib.ce_multi_get_state(self._h, theta.ctypes.data, step.ctypes.data),
              'ce_multi_get_state')
        return {'theta': theta, 'step': step}

    def close(self):
        if getattr(self, '_h', None):
            self._lib.ce_multi_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass
