"""CPU oracle for the Optimize-v0 hot path -- TEST INFRASTRUCTURE ONLY.

This package is a plain-numpy (float64) restatement of the reference's
per-step dynamics, used as the *checker* by ``tests/``,
``__graft_entry__.smoke()`` and the ``cpu_baseline`` leg of ``bench.py``.
Nothing in ``custom_envs_amd`` imports it; the product path runs the HIP
engine and fails loudly when that engine is missing.

Modules
-------
seeding      old-gym ``gym.utils.seeding.np_random`` restated (third-party,
             absent here -- parity of seed -> stream is *unpinned*, see
             DESIGN.md section "Oracle").
optimize     ``custom_envs/envs/optimize.py`` + ``baseenvironment.py`` +
             the missing ``custom_envs.models.ModelNumpy`` (build-defined,
             SURVEY.md section 8a row A7) + ``InMemoryDataSet`` shims.
vectorize    ``custom_envs/vectorize/concurrentvecenv.py`` restated: one
             worker (thread or process) + one ``multiprocessing.Pipe`` per
             env, pickled command loop, ``np.stack`` in ``step_wait``.
data         the synthetic datasets the configs name.

Pinning: the reference's importable pieces (``utils_common.shuffle``,
``to_onehot``, ``History``) are cross-checked in ``tests/test_oracle.py``
when ``/root/reference`` is present; golden fixtures generated from this
oracle live in ``tests/golden`` (script: ``oracle/gen_golden.py``).
"""
