"""ORACLE — test infrastructure, never product code.

CPU restatements (numpy) of the CB-Whisper hot path, each function citing the
reference file:line it follows.  Parity of these restatements is pinned by
fixtures generated from the reference's own modules (``tests/golden/``).
Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s cpu_baseline
leg may import anything under ``oracle/``.
"""
import os
import sys

_pkg = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "enhance-cb-whisper_amd")
if _pkg not in sys.path:  # topology tables (cbw.synth) only; no compute from the product
    sys.path.insert(0, _pkg)
