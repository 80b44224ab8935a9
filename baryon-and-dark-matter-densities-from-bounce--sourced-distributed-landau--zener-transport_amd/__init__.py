"""lzq: MI355X-native engine for the bounce-sourced Landau-Zener yield hot path of
SFVdSB first_principles_yields.py (KJMA A/V kernel, Y_B direct quadrature, LZ probability,
density epilogue, parameter sweeps over 1-8 GPUs).  See DESIGN.md.

Importing the package does not touch the GPU; `Engine()` does.
"""
from . import _native, build, config  # noqa: F401
from .config import Config, default_config, load_config, write_template  # noqa: F401

__all__ = ["Config", "default_config", "load_config", "write_template", "Engine", "BoltzmannSystem",
           "AoverVKernel"]
__version__ = "0.1.0"


def __getattr__(name):  # lazy: torch is only imported when the engine is used
    if name == "Engine":
        from .engine import Engine
        return Engine
    if name in ("BoltzmannSystem", "AoverVKernel"):
        from . import boltzmann
        return getattr(boltzmann, name)
    raise AttributeError(name)
