"""CPU restatement of the reference metric path -- TEST INFRASTRUCTURE ONLY.

Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s cpu_baseline
leg may import this package, and only as the checker or the timed CPU
baseline.  The product (``sctools_amd``) never imports it.
"""
