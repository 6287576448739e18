"""Import (building on first use if needed) the C++ host runtime `_runtime`."""
from __future__ import annotations

import importlib

_mod = None


def load():
    global _mod
    if _mod is not None:
        return _mod
    try:
        _mod = importlib.import_module("aws_k8s_ansible_provisioner_amd._runtime")
    except ImportError:
        from . import build_ext

        build_ext.build_runtime()
        _mod = importlib.import_module("aws_k8s_ansible_provisioner_amd._runtime")
    return _mod
