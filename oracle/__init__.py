"""ORACLE -- CPU restatement of the reference hot path (test infrastructure ONLY).

Only ``tests/``, ``__graft_entry__.smoke()`` and the ``cpu_baseline`` leg of ``bench.py``
may import this package.  The product path (``distributed_aerial_transportation_amd``)
never imports it and fails loudly when its HIP library is missing.
"""
