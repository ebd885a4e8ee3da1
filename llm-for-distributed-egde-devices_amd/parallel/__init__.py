"""Distributed execution: layer-partitioned pipeline over RCCL point-to-point (see pipeline.py)."""
