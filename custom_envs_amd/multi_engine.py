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
from custom_envs_amd.engine import check_rollout

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
            raise RuntimeError('Not a name of a problem: %r' % problem)
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
        if ndims > _native.CE_MULTI_MAX_PARAMS:
            raise ValueError('MultiOptLRs function problems run up to %d dimensions (one lane per '
                             'agent, an env within one wave); got %d'
                             % (_native.CE_MULTI_MAX_PARAMS, ndims))
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
        self._lib, self._h, self._prefix = lib, handle, 'ce_multi_'
        self._bind_outputs()
        self.many_kernel = lib.ce_multi_step_many_kernel(handle).decode()

    # ------------------------------------------------- K steps in one launch
    def set_persistent(self, on=True):
        """K-step calls as ONE launch of multi_persist_kernel (max_history 5)
        or one launch per step (on=False, the A/B form)."""
        self._call('set_persistent', 1 if on else 0)
        self.many_kernel = self._lib.ce_multi_step_many_kernel(self._h).decode()

    @property
    def persistent(self):
        return self.many_kernel.startswith('multi_persist')

    def alloc_rollout(self, k, torch_device=None):
        """[k] output records (256-B aligned field segments per record):
        (fields, record_bytes), fields[name] a (k, rows, ...) view."""
        import torch
        from custom_envs_amd.distributed import PackedLayout
        lay = PackedLayout(self.output_fields(), self.num_envs)
        buf = torch.zeros(int(k) * lay.nbytes, dtype=torch.uint8,
                          device=torch_device or torch.device('cuda'))
        fields = lay.chunk_views(buf, self.num_envs, int(k))
        fields['_buffer'] = buf
        return fields, lay.nbytes

    def rollout_device(self, k, actions, fields, record_bytes, per_step_actions=True):
        """k steps; step t reads actions[t] and writes record t of ``fields``
        (ce_multi_step_many_strided).  ``fields`` must hold at least k
        records of ``record_bytes`` each (``engine.check_rollout``)."""
        first = check_rollout(self.output_fields(), self.num_envs, k, actions, self.rows, fields,
                              record_bytes, per_step_actions)
        o = self._outputs(first)
        stride = self.rows if per_step_actions else 0
        self._call('step_many_strided', int(k), actions.data_ptr(), stride, ctypes.byref(o),
                   int(record_bytes))

    def rollout_runner(self, k, actions, fields, record_bytes, per_step_actions=True):
        """rollout_device bound once."""
        first = check_rollout(self.output_fields(), self.num_envs, k, actions, self.rows, fields,
                              record_bytes, per_step_actions)
        o = self._outputs(first)
        fn, h, ap, ref = self._fn('step_many_strided'), self._h, actions.data_ptr(), ctypes.byref(o)
        kk, stride, rb = int(k), (self.rows if per_step_actions else 0), int(record_bytes)

        def run():
            rc = fn(h, kk, ap, stride, ref, rb)
            if rc:
                check(rc, self._prefix + 'step_many_strided')
        run.keep = (actions, fields, o)
        return run

    def _fn(self, name):
        return getattr(self._lib, self._prefix + name)

    def _call(self, name, *args):
        return check(self._fn(name)(self._h, *args), self._prefix + name)

    def _bind_outputs(self):
        self.row_agents = row_agents(self.n_params)
        view = CeMultiOutputs()
        self._call('host_outputs', ctypes.byref(view))
        E, P, W = self.num_envs, self.n_params, 3 * self.max_history
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
        self._call('reset', None, 0)
        return self._host['obs'].copy()

    def step_async(self, actions):
        actions = np.ascontiguousarray(actions, dtype=np.float32).reshape(self.rows)
        self._pending = actions
        self._call('step_async', actions.ctypes.data, None, 0)

    def step_wait(self):
        self._call('wait')
        self._pending = None
        return self._host

    def step(self, actions):
        self.step_async(actions)
        return self.step_wait()

    # ------------------------------------------------------------- device mode
    def set_stream(self, stream_handle):
        self._call('set_stream', ctypes.c_void_p(stream_handle or 0))

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
        self._call('reset', ctypes.byref(o), _native.CE_PTR_DEVICE)

    def step_device(self, actions, out):
        if actions.numel() < self.rows or not actions.is_contiguous():
            raise ValueError('actions must be a contiguous float32 tensor of E*P rows')
        o = self._outputs(out)
        self._call('step_async', actions.data_ptr(), ctypes.byref(o), _native.CE_PTR_DEVICE)

    def step_many_device(self, k, actions, out, per_step_actions=True):
        if actions.numel() < (k if per_step_actions else 1) * self.rows:
            raise ValueError('actions tensor too small')
        o = self._outputs(out)
        stride = self.rows if per_step_actions else 0
        self._call('step_many', int(k), actions.data_ptr(), stride, ctypes.byref(o))

    def prepare_many_device(self, k, actions, out, per_step_actions=True):
        """Instantiate (and upload) the k-step hipGraph without running it."""
        if actions.numel() < (k if per_step_actions else 1) * self.rows:
            raise ValueError('actions tensor too small')
        o = self._outputs(out)
        stride = self.rows if per_step_actions else 0
        self._call('step_many_prepare', int(k), actions.data_ptr(), stride, ctypes.byref(o))

    def wait(self):
        self._call('wait')

    def get_state(self):
        theta = np.zeros((self.num_envs, self.n_params), np.float32)
        step = np.zeros(self.num_envs, np.int32)
        check(self._lib.ce_multi_get_state(self._h, theta.ctypes.data, step.ctypes.data),
              'ce_multi_get_state')
        return {'theta': theta, 'step': step}

    def close(self):
        if getattr(self, '_h', None):
            self._fn('destroy')(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


# create_neural_net's default layers (custom_envs/utils/utils_tf.py:74) and
# load_data's default set + batch size (custom_envs/data/load_data.py:47);
# 'iris' is a git-LFS pointer in the reference, so its iris-shaped stand-in
NN_DEFAULT_HIDDEN = (256, 256)
NN_DEFAULT_DATA = 'iris_synthetic'


def resolve_nn(data_set=None, hidden=None):
    """(features float32 [N][F], labels int32 [N], K, batch size, hidden)."""
    if data_set is None:
        from custom_envs_amd.data import load_data
        data_set = load_data(NN_DEFAULT_DATA, batch_size=32)
    features = np.ascontiguousarray(data_set.features, dtype=np.float32)
    targets = np.asarray(data_set.targets)
    if features.ndim != 2 or targets.ndim != 2:
        raise ValueError('the network problem needs (N, F) features and one-hot (N, K) targets')
    labels = np.ascontiguousarray(np.argmax(targets, axis=1), dtype=np.int32)
    hidden = tuple(int(h) for h in (NN_DEFAULT_HIDDEN if hidden is None else hidden))
    return features, labels, targets.shape[1], int(data_set.batch_size), hidden


class NNMultiEngine(MultiOptEngine):
    """E MultiOptLRs envs over the OptimizeNN problem (get_problem('nn'),
    custom_envs/problems/__init__.py:7-16): one agent per network parameter,
    P = sum of the layers' kernel and bias sizes.  Seeds default to the env
    index (the reference seeds each env from os.urandom, baseenvironment.py:17)."""

    def __init__(self, num_envs, data_set=None, hidden=None, max_batches=400, max_history=5,
                 device=0, auto_reset=True, seeds=None):
        lib = _native.load()
        features, labels, K, B, hidden = resolve_nn(data_set, hidden)
        self.num_envs = int(num_envs)
        self.max_history, self.max_batches = int(max_history), int(max_batches)
        self.hidden, self.n_features, self.n_classes = hidden, features.shape[1], K
        self.batch_size, self.n_rows = B, features.shape[0]
        if len(hidden) > _native.CE_NN_MAX_HIDDEN:
            raise _native.NativeEngineError('at most %d hidden layers' % _native.CE_NN_MAX_HIDDEN)
        cfg = _native.CeNnConfig(abi_version=_native.ABI_VERSION, device=int(device),
                                 num_envs=self.num_envs, n_rows=features.shape[0],
                                 n_features=features.shape[1], n_classes=K, batch_size=B,
                                 n_hidden=len(hidden), max_history=self.max_history,
                                 max_batches=self.max_batches, auto_reset=1 if auto_reset else 0)
        for i, w in enumerate(hidden):
            cfg.hidden[i] = w
        handle = ctypes.c_void_p()
        check(lib.ce_nn_create(ctypes.byref(cfg), features.ctypes.data, labels.ctypes.data,
                               ctypes.byref(handle)), 'ce_nn_create')
        self._lib, self._h, self._prefix = lib, handle, 'ce_nn_'
        self.n_params = int(lib.ce_nn_n_params(handle))
        self._bind_outputs()
        self.seed(seeds)
        self.many_kernel = 'nn_* (one launch sequence per step)'

    def set_persistent(self, on=True):
        if on:
            raise _native.NativeEngineError('the network problem has no K-step launch form')

    def rollout_device(self, *args, **kwargs):
        raise _native.NativeEngineError('the network problem has no strided K-step form')

    rollout_runner = rollout_device

    @property
    def dims(self):
        return (self.n_features,) + self.hidden + (self.n_classes,)

    def seed(self, seeds=None):
        """seeds[i] seeds env i as gym.utils.seeding.np_random(seeds[i])
        (baseenvironment.py:20-28): the reset's initial weights and shuffle,
        and the epoch-end shuffle."""
        if seeds is None:
            seeds = range(self.num_envs)
        arr = np.ascontiguousarray([int(s) % (1 << 64) for s in seeds], dtype=np.uint64)
        if arr.size != self.num_envs:
            raise ValueError('one seed per env')
        self._call('seed', arr.ctypes.data, int(arr.size))
        self.seeds = [int(v) for v in arr]       # the current per-env seeds
        return list(self.seeds)

    def get_state(self):
        E, P, N = self.num_envs, self.n_params, self.n_rows
        st = {'theta': np.zeros((E, P), np.float32), 'gprev': np.zeros((E, P), np.float32),
              'step': np.zeros(E, np.int32), 'cursor': np.zeros(E, np.int32),
              'order': np.zeros((E, N), np.int32)}
        self._call('get_state', *(st[k].ctypes.data for k in
                                  ('theta', 'gprev', 'step', 'cursor', 'order')))
        return st


def create_engine(num_envs, problem='func', **kwargs):
    """The engine a MultiOptLRs spec runs on: 'nn' -> NNMultiEngine, else the
    function problems."""
    if problem == 'nn':
        kwargs.pop('initial_points', None)
        return NNMultiEngine(num_envs, **kwargs)
    kwargs.pop('data_set', None)
    kwargs.pop('hidden', None)
    return MultiOptEngine(num_envs, problem, **kwargs)
