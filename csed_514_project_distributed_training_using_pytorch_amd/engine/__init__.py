"""Training engines: fused LeNet (two HIP launches / step), modular (per-op), CLIs.

Import the submodules directly (``engine.fused``, ``engine.modular``,
``engine.cli``); nothing is imported eagerly here.
"""
