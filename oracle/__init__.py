"""CPU oracle for the mobile-env step hot path -- TEST INFRASTRUCTURE ONLY.

Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline`` leg may import
anything from this package, and only as the checker / the timed CPU baseline. The product
(``mobile-env-gan_amd/``) never imports it and has no CPU fallback.

* ``oracle.vec``  -- NumPy restatement of ``MComCore.reset/step`` (reference
  ``mobile_env/core/base.py:172-296``), vectorised across independent envs, sequential per env
  where the reference is (the PCG64 draw order). Pinned bit-for-bit against the golden fixtures
  in ``tests/golden/`` (generated from the reference itself by ``tests/golden/make_golden.py``)
  and against the two notebook snapshots.
* ``oracle.port`` -- per-object pure-Python restatement with the reference's structure (entity
  objects, plugin objects, dict/set bookkeeping, per-pair channel evaluation); slow, used for
  small parity cases and as the ``cpu_baseline`` ("port") in ``bench.py``.

Parity status: PINNED (fixtures from the reference run in the dev container).
"""
