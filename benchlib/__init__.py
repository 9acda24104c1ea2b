"""bench.py's helpers, modes and companion runs (split out of bench.py)."""
