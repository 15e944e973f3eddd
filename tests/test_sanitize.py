"""Host code under AddressSanitizer + UndefinedBehaviorSanitizer (SURVEY 5,
"race detection / sanitizers"): the engine's sources built with the
sanitizers on the host side only (tests/sanitize/build.py), driving every
host-only entry point (seeding.cpp: SHA-512, MT19937, the legacy gauss /
uniform / shuffle draws) over edge seeds and shapes, and the argument
validation of every C-ABI entry point (ce_create's checks and the network
geometry's included).  A sanitizer report aborts the driver; the draws it
prints must equal the numpy oracle's.  CPU only: no GPU call succeeds here.
"""
import os
import subprocess
import sys

import numpy as np
import pytest

from conftest import ROOT

sys.path.insert(0, os.path.join(ROOT, 'tests', 'sanitize'))


def _parse(text):
    seeds, cur = {}, None
    for line in text.splitlines():
        tag, *vals = line.split()
        if tag == 'seed':
            cur = seeds.setdefault(int(vals[0]), {})
        elif cur is not None and tag not in ('failures',):
            cur[tag] = [int(v, 16) for v in vals]
    return seeds


def test_host_code_under_asan_ubsan():
    import build as sbuild
    try:
        driver = sbuild.build()
    except Exception as exc:       # pragma: no cover - toolchain missing
        pytest.fail('sanitizer build failed: %s' % exc)
    env = dict(os.environ, ASAN_OPTIONS='detect_leaks=0:halt_on_error=1:abort_on_error=0',
               UBSAN_OPTIONS='halt_on_error=1:print_stacktrace=1')
    env.pop('LD_PRELOAD', None) if env.get('LD_PRELOAD', '').find('asan') >= 0 else None
    proc = subprocess.run([driver], capture_output=True, text=True, env=env, timeout=300)
    assert proc.returncode == 0, proc.stderr[-3000:]
    assert 'runtime error' not in proc.stderr and 'AddressSanitizer' not in proc.stderr
    assert proc.stdout.strip().endswith('failures 0')
    from oracle.multinn import nn_draws
    from oracle.optimize import initial_draws, initial_draws_mlp
    draws = _parse(proc.stdout)
    assert sorted(draws) == [0, 3, 2**31 - 1, 2**33, 2**64 - 1]
    for seed, d in draws.items():
        w, p = initial_draws(seed, 10, 2, 256)
        assert np.array_equal(np.array(d['lr_w'], np.uint64).view(np.float64), w.ravel())
        assert np.array_equal(d['lr_p'], p)
        w, p = initial_draws_mlp(seed, 24, 64, 10, 200)
        assert np.array_equal(np.array(d['mlp_w'], np.uint32).view(np.float32), w)
        assert np.array_equal(d['mlp_p'], p)
        w, rp, ep = nn_draws(seed, (4, 32, 3), 150)
        assert np.array_equal(np.array(d['nn_w'], np.uint32).view(np.float32), w)
        assert np.array_equal(d['nn_rp'], rp) and np.array_equal(d['nn_ep'], ep)
