"""Utilities: flat parameter storage, checkpoints, log formats, plots, profiling."""
from . import checkpoint, flat, metrics, plot, prof  # noqa: F401
