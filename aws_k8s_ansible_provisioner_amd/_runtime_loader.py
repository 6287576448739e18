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
    from . import build_ext

    try:
        mod = importlib.import_module("aws_k8s_ansible_provisioner_amd._runtime")
    except ImportError:
        build_ext.build_runtime()
        mod = importlib.import_module("aws_k8s_ansible_provisioner_amd._runtime")
    # provenance: the module must be built from the runtime sources beside it
    have = mod.build_hash() if hasattr(mod, "build_hash") else "none"
    want = build_ext.runtime_tree_hash()
    if have != want and os.environ.get("AKAP_ALLOW_STALE_NATIVE") != "1":
        raise ImportError(f"_runtime was built from other sources ({have[:16]} vs {want[:16]}): "
                          "rebuild with python -m aws_k8s_ansible_provisioner_amd.build_ext")
    _mod = mod
    return _mod
