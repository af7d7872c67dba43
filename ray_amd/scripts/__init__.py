"""Command line entry points: ``python -m ray_amd.scripts <command>``."""
