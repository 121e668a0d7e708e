"""ORACLE — test infrastructure only (CPU restatement of the reference maths).

Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline`` leg may
import this package, and only as the checker / the timed CPU baseline — never as the
product path. The product (``magic_amd``) never imports it.
"""
