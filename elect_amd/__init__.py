"""elect_amd — MI355X-native Reed-Solomon engine for ELECT's redundancy-transitioning path.

  elect_amd.coder   Java coder API mirror (NativeRSEncoder / NativeRSDecoder, ...)
  elect_amd.batch   device-resident batched encode / decode / update over torch tensors
  elect_amd._lib    ctypes binding of libelect_ec.so (include/elect_ec.h)
  elect_amd.build   hipcc recipe for libelect_ec.so

Submodules are imported lazily so `python -m elect_amd.build` works before the
library exists; importing anything that computes without the library raises.
"""
import importlib

__all__ = ["coder", "batch", "build", "RSCoder", "NativeRSEncoder", "NativeRSDecoder",
           "ErasureCoderOptions", "ByteBuffer"]

_LAZY = {
    "RSCoder": "coder",
    "NativeRSEncoder": "coder",
    "NativeRSDecoder": "coder",
    "ErasureCoderOptions": "coder",
    "ByteBuffer": "coder",
}


def __getattr__(name):
    if name in ("coder", "batch", "build", "_lib"):
        return importlib.import_module(f"{__name__}.{name}")
    if name in _LAZY:
        return getattr(importlib.import_module(f"{__name__}.{_LAZY[name]}"), name)
    raise AttributeError(name)
