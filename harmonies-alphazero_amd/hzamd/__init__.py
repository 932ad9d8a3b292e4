"""hzamd — MI355X-native Harmonies self-play engine (host side).

The compute lives in libhz.so (HIP kernels for gfx950, C-ABI in
include/hz_abi.h); this package binds it and mirrors the reference's Python
surfaces.  The drop-in modules harmonies_engine / process_game_state / MCTS
sit next to this package (put harmonies-alphazero_amd/ on sys.path).
"""
from . import state  # noqa: F401

__all__ = ["state", "env", "BatchedEnv"]


def __getattr__(name):
    if name == "BatchedEnv":
        from .env import BatchedEnv
        return BatchedEnv
    if name == "env":
        from . import env
        return env
    raise AttributeError(name)
