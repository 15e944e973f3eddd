"""engine.check_rollout, the host-side guard of the strided K-step calls
(ADVICE r05): what it refuses before any pointer reaches a kernel.  The
checks that need device tensors run in tests/test_gpu_persist.py and
tests/test_gpu_multi.py; here the CPU-tensor cases and the spec logic."""
import pytest

torch = pytest.importorskip('torch')

from custom_envs_amd.engine import check_rollout  # noqa: E402

SPEC = [('obs', torch.float32, 1, (41,)), ('reward', torch.float32, 1, ()),
        ('episode_len', torch.int32, 1, ())]


def _fields(k, E=8):
    return {'obs': torch.zeros((k, E, 41)), 'reward': torch.zeros((k, E)),
            'episode_len': torch.zeros((k, E), dtype=torch.int32)}


def test_host_actions_are_refused():
    with pytest.raises(ValueError, match='device tensor'):
        check_rollout(SPEC, 8, 2, torch.zeros((2, 8, 20)), 160, _fields(2), 0)


def test_nonpositive_k_is_refused():
    with pytest.raises(ValueError, match='k must be'):
        check_rollout(SPEC, 8, 0, torch.zeros((2, 8, 20)), 160, _fields(2), 0)


def test_float64_actions_are_refused():
    with pytest.raises(ValueError, match='float32'):
        check_rollout(SPEC, 8, 1, torch.zeros((1, 8, 20), dtype=torch.float64), 160, _fields(1), 0)
