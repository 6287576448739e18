"""Import (building on first use if needed) the C++ host runtime `_runtime`.

AKAP_RUNTIME_DIR=<dir> imports the `_runtime` extension from <dir> instead of the package
(the ASan/UBSan build of tools/sanitize_runtime.sh)."""
from __future__ import annotations

import importlib
import os
import sys

_mod = None


def load():
    global _mod
    if _mod is not None:
        return _mod
    alt = os.environ.get("AKAP_RUNTIME_DIR")
    if alt:
        sys.path.insert(0, alt)
        _mod = importlib.import_module("_runtime")
        return _mod
    try:
        _mod = importlib.import_module("aws_k8s_ansible_provisioner_amd._runtime")
    except ImportError:
        from . import build_ext

        build_ext.build_runtime()
        _mod = importlib.import_module("aws_k8s_ansible_provisioner_amd._runtime")
    return _mod
