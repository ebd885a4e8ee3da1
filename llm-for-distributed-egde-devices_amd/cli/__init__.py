"""Command-line entry points (reference-compatible flags): evaluate, combine, cpu_int8, serve,
quantize, pipeline, fetch.  Run as ``python -m edgellm.cli.<name>``."""
