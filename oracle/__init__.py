"""CPU oracle for the TRPO update engine — test infrastructure only.

Imported only by ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s
``cpu_baseline`` leg.  Never imported by ``trpo_amd`` (the product).
"""
