"""MI355X-native hot path of distributed-lab/linea-stark-prover.

The product is ``_lib/liblsp_hip.so`` (HIP kernels for gfx950 + C++ host
orchestration behind the C-ABI of ``include/lsp.h``).  This package is the
Python-side mirror of the reference's plug point (bin/src/config.rs:9-25):
``prover`` (Dft / Mmcs / FriFolder / prove / verify), ``air`` (the AirConfig
list of LineaAIR), ``field`` (element-array helpers).
"""
from . import air, field  # noqa: F401
from ._lib import LIB_PATH, LspError, lib  # noqa: F401


def __getattr__(name):
    # lazy: importing the prover API loads the HIP library
    if name in ("prover",):
        import importlib
        return importlib.import_module(f".{name}", __name__)
    raise AttributeError(name)
