"""ctypes binding of the HIP engine (include/custom_envs_amd.h).

The product path has no CPU fallback: if the in-tree library is missing or
cannot be loaded, importing the engine raises ``NativeEngineError``.
"""
import ctypes
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_HERE, 'lib', 'libcustom_envs_amd.so')
# CE_LIB=diag selects the phase-stamped profiling build (same ABI + ce_diag_stamps)
# CE_LIB=<name> selects lib/libcustom_envs_amd_<name>.so (experiment builds).
if os.environ.get('CE_LIB') == 'diag':
    # never pushed to the GPU box (.gpurunignore): built there from the
    # sources, so a stale diagnostic library cannot load
    LIB_PATH = os.path.join(_HERE, 'lib', 'libcustom_envs_amd_diag.so')
elif os.environ.get('CE_LIB'):
    LIB_PATH = os.path.join(_HERE, 'lib', 'libcustom_envs_amd_%s.so' % os.environ['CE_LIB'])

ABI_VERSION = 5
CE_OK, CE_EINVAL, CE_EHIP, CE_ENOMEM, CE_ESTATE, CE_EUNSUPPORTED = 0, -1, -2, -3, -4, -5
CE_PROBLEM_SOFTMAX, CE_PROBLEM_MLP = 0, 1
CE_F64, CE_F32 = 0, 1
CE_PTR_DEVICE = 1

STATUS_NAMES = {CE_EINVAL: 'CE_EINVAL', CE_EHIP: 'CE_EHIP', CE_ENOMEM: 'CE_ENOMEM',
                CE_ESTATE: 'CE_ESTATE', CE_EUNSUPPORTED: 'CE_EUNSUPPORTED'}

# Every symbol include/custom_envs_amd.h declares.
EXPORTS = (
    'ce_abi_version', 'ce_last_error', 'ce_stale_error_count', 'ce_stale_error_note', 'ce_create', 'ce_destroy', 'ce_set_stream',
    'ce_set_compact_outputs', 'ce_num_envs', 'ce_obs_dim', 'ce_act_dim', 'ce_seed', 'ce_seed_draws',
    'ce_seed_draws_mlp', 'ce_reset',
    'ce_step', 'ce_step_async', 'ce_wait', 'ce_step_many', 'ce_step_many_prepare',
    'ce_step_many_strided', 'ce_set_persistent', 'ce_step_many_kernel',
    'ce_host_outputs', 'ce_step_kernel',
    'ce_get_state', 'ce_set_state',
    'ce_multi_create', 'ce_multi_destroy', 'ce_multi_set_stream', 'ce_multi_reset',
    'ce_multi_step', 'ce_multi_step_async', 'ce_multi_wait', 'ce_multi_step_many',
    'ce_multi_step_many_prepare', 'ce_multi_step_many_strided', 'ce_multi_set_persistent',
    'ce_multi_step_many_kernel',
    'ce_multi_host_outputs', 'ce_multi_get_state',
    'ce_nn_create', 'ce_nn_destroy', 'ce_nn_set_stream', 'ce_nn_n_params', 'ce_nn_seed',
    'ce_nn_seed_draws', 'ce_nn_reset', 'ce_nn_step', 'ce_nn_step_async', 'ce_nn_wait',
    'ce_nn_step_many', 'ce_nn_step_many_prepare', 'ce_nn_host_outputs', 'ce_nn_get_state',
)

CE_FUNC_ROSENBROCK_PAIRS = 0
CE_MULTI_MAX_PARAMS = 64
MULTI_INFO_KEYS = ('loss', 'batch_loss', 'weights_mean', 'weights_sum', 'actions_mean',
                   'actions_std', 'states_mean', 'states_sum', 'grads_mean', 'grads_sum',
                   'loss_mean', 'adjusted_loss', 'adjusted_grad', 'grad_diff')


class NativeEngineError(RuntimeError):
    """Raised when the HIP engine is missing or a C-ABI call fails."""


class CeConfig(ctypes.Structure):
    _fields_ = [(name, ctypes.c_int32) for name in (
        'abi_version', 'problem', 'precision', 'device', 'num_envs', 'n_rows',
        'n_features', 'n_classes', 'batch_size', 'max_steps', 'auto_reset', 'n_hidden',
        'n_layers')] + [('hidden', ctypes.c_int32 * 4)]


class CeOutputs(ctypes.Structure):
    _fields_ = [('obs', ctypes.c_void_p), ('reward', ctypes.c_void_p),
                ('done', ctypes.c_void_p), ('objective', ctypes.c_void_p),
                ('accuracy', ctypes.c_void_p), ('episode_len', ctypes.c_void_p)]


class CeMultiConfig(ctypes.Structure):
    _fields_ = [(name, ctypes.c_int32) for name in (
        'abi_version', 'device', 'num_envs', 'n_params', 'function', 'max_history',
        'max_batches', 'auto_reset')] + [('initial_points', ctypes.c_float * CE_MULTI_MAX_PARAMS)]


class CeMultiOutputs(ctypes.Structure):
    _fields_ = [('obs', ctypes.c_void_p), ('reward', ctypes.c_void_p),
                ('done', ctypes.c_void_p), ('info', ctypes.c_void_p),
                ('episode_len', ctypes.c_void_p)]


CE_NN_MAX_HIDDEN = 4


class CeNnConfig(ctypes.Structure):
    _fields_ = ([(name, ctypes.c_int32) for name in (
        'abi_version', 'device', 'num_envs', 'n_rows', 'n_features', 'n_classes',
        'batch_size', 'n_hidden')] + [('hidden', ctypes.c_int32 * CE_NN_MAX_HIDDEN)] +
        [(name, ctypes.c_int32) for name in ('max_history', 'max_batches', 'auto_reset')])


class CeState(ctypes.Structure):
    _fields_ = [('weights', ctypes.c_void_p), ('grad_hist', ctypes.c_void_p),
                ('loss_hist', ctypes.c_void_p), ('step', ctypes.c_void_p),
                ('init_weights', ctypes.c_void_p), ('order', ctypes.c_void_p)]


_lib = None


def _declare(lib):
    vp, i32, u32, i64 = ctypes.c_void_p, ctypes.c_int32, ctypes.c_uint32, ctypes.c_int64
    sig = {
        'ce_abi_version': ([], ctypes.c_int),
        'ce_last_error': ([], ctypes.c_char_p),
        'ce_stale_error_count': ([], ctypes.c_int64),
        'ce_stale_error_note': ([], ctypes.c_char_p),
        'ce_create': ([ctypes.POINTER(CeConfig), vp, vp, ctypes.POINTER(vp)], ctypes.c_int),
        'ce_destroy': ([vp], None),
        'ce_set_stream': ([vp, vp], ctypes.c_int),
        'ce_set_compact_outputs': ([vp, i32], ctypes.c_int),
        'ce_num_envs': ([vp], ctypes.c_int),
        'ce_obs_dim': ([vp], ctypes.c_int),
        'ce_act_dim': ([vp], ctypes.c_int),
        'ce_seed': ([vp, vp, i32], ctypes.c_int),
        'ce_seed_draws': ([ctypes.c_uint64, i32, i32, i32, vp, vp], ctypes.c_int),
        'ce_seed_draws_mlp': ([ctypes.c_uint64, i32, i32, i32, i32, vp, vp], ctypes.c_int),
        'ce_reset': ([vp, ctypes.POINTER(CeOutputs), u32], ctypes.c_int),
        'ce_step': ([vp, vp, ctypes.POINTER(CeOutputs), u32], ctypes.c_int),
        'ce_step_async': ([vp, vp, ctypes.POINTER(CeOutputs), u32], ctypes.c_int),
        'ce_wait': ([vp], ctypes.c_int),
        'ce_step_many': ([vp, i32, vp, i64, ctypes.POINTER(CeOutputs)], ctypes.c_int),
        'ce_step_many_prepare': ([vp, i32, vp, i64, ctypes.POINTER(CeOutputs)], ctypes.c_int),
        'ce_step_many_strided': ([vp, i32, vp, i64, ctypes.POINTER(CeOutputs), i64], ctypes.c_int),
        'ce_set_persistent': ([vp, i32], ctypes.c_int),
        'ce_step_many_kernel': ([vp], ctypes.c_char_p),
        'ce_host_outputs': ([vp, ctypes.POINTER(CeOutputs)], ctypes.c_int),
        'ce_step_kernel': ([vp], ctypes.c_char_p),
        'ce_get_state': ([vp, ctypes.POINTER(CeState)], ctypes.c_int),
        'ce_set_state': ([vp, ctypes.POINTER(CeState)], ctypes.c_int),
        'ce_multi_create': ([ctypes.POINTER(CeMultiConfig), ctypes.POINTER(vp)], ctypes.c_int),
        'ce_multi_destroy': ([vp], None),
        'ce_multi_set_stream': ([vp, vp], ctypes.c_int),
        'ce_multi_reset': ([vp, ctypes.POINTER(CeMultiOutputs), u32], ctypes.c_int),
        'ce_multi_step': ([vp, vp, ctypes.POINTER(CeMultiOutputs), u32], ctypes.c_int),
        'ce_multi_step_async': ([vp, vp, ctypes.POINTER(CeMultiOutputs), u32], ctypes.c_int),
        'ce_multi_wait': ([vp], ctypes.c_int),
        'ce_multi_step_many': ([vp, i32, vp, i64, ctypes.POINTER(CeMultiOutputs)], ctypes.c_int),
        'ce_multi_step_many_prepare': ([vp, i32, vp, i64, ctypes.POINTER(CeMultiOutputs)],
                                       ctypes.c_int),
        'ce_multi_step_many_strided': ([vp, i32, vp, i64, ctypes.POINTER(CeMultiOutputs), i64],
                                       ctypes.c_int),
        'ce_multi_set_persistent': ([vp, i32], ctypes.c_int),
        'ce_multi_step_many_kernel': ([vp], ctypes.c_char_p),
        'ce_multi_host_outputs': ([vp, ctypes.POINTER(CeMultiOutputs)], ctypes.c_int),
        'ce_multi_get_state': ([vp, vp, vp], ctypes.c_int),
        'ce_nn_create': ([ctypes.POINTER(CeNnConfig), vp, vp, ctypes.POINTER(vp)], ctypes.c_int),
        'ce_nn_destroy': ([vp], None),
        'ce_nn_set_stream': ([vp, vp], ctypes.c_int),
        'ce_nn_n_params': ([vp], ctypes.c_int),
        'ce_nn_seed': ([vp, vp, i32], ctypes.c_int),
        'ce_nn_seed_draws': ([ctypes.c_uint64, i32, vp, i32, vp, vp, vp], ctypes.c_int),
        'ce_nn_reset': ([vp, ctypes.POINTER(CeMultiOutputs), u32], ctypes.c_int),
        'ce_nn_step': ([vp, vp, ctypes.POINTER(CeMultiOutputs), u32], ctypes.c_int),
        'ce_nn_step_async': ([vp, vp, ctypes.POINTER(CeMultiOutputs), u32], ctypes.c_int),
        'ce_nn_wait': ([vp], ctypes.c_int),
        'ce_nn_step_many': ([vp, i32, vp, i64, ctypes.POINTER(CeMultiOutputs)], ctypes.c_int),
        'ce_nn_step_many_prepare': ([vp, i32, vp, i64, ctypes.POINTER(CeMultiOutputs)],
                                    ctypes.c_int),
        'ce_nn_host_outputs': ([vp, ctypes.POINTER(CeMultiOutputs)], ctypes.c_int),
        'ce_nn_get_state': ([vp, vp, vp, vp, vp, vp], ctypes.c_int),
    }
    for name, (args, res) in sig.items():
        fn = getattr(lib, name)
        fn.argtypes = args
        fn.restype = res


def load():
    """Load the in-tree engine library (no fallback)."""
    global _lib
    if _lib is None:
        if os.environ.get('CE_LIB') == 'diag':
            from custom_envs_amd import build as _build
            _build.build(diag=True)          # rebuilt unless newer than every source
        if not os.path.exists(LIB_PATH):
            raise NativeEngineError(
                'HIP engine library not built: %s (run python -m custom_envs_amd.build)'
                % LIB_PATH)
        try:
            lib = ctypes.CDLL(LIB_PATH)
        except OSError as err:
            raise NativeEngineError('cannot load %s: %s' % (LIB_PATH, err)) from err
        _declare(lib)
        if lib.ce_abi_version() != ABI_VERSION:
            raise NativeEngineError('engine ABI mismatch')
        _lib = lib
    return _lib


def check(rc, what):
    if rc != CE_OK:
        msg = load().ce_last_error().decode(errors='replace')
        raise NativeEngineError('%s: %s (%s)' % (what, msg, STATUS_NAMES.get(rc, rc)))
    return rc


_stale_seen = [0]


def warn_stale():
    """Warn (once per new batch) when an entry point found a sticky HIP error
    pending that an earlier, unrelated operation left behind and cleared it
    (ce_stale_error_count / ce_stale_error_note): the failure is reported, not
    lost.  Returns the process-wide count."""
    lib = load()
    n = int(lib.ce_stale_error_count())
    if n > _stale_seen[0]:
        import warnings
        note = lib.ce_stale_error_note().decode(errors='replace')
        warnings.warn('custom_envs_amd: %d stale HIP error(s) found pending and cleared; last: %s'
                      % (n - _stale_seen[0], note), RuntimeWarning, stacklevel=2)
        _stale_seen[0] = n
    return n
