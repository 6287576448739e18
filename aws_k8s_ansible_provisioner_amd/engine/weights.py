"""Checkpoint loading from a local directory (the model PVC): safetensors only --
no pickle-based formats are ever deserialised."""
from __future__ import annotations

import glob
import os


def load_safetensors_dir(path: str, device: str = "cpu") -> dict:
    from safetensors.torch import load_file

    files = sorted(glob.glob(os.path.join(path, "*.safetensors")))
    if not files:
        raise FileNotFoundError(f"no *.safetensors under {path}")
    sd: dict = {}
    for f in files:
        sd.update(load_file(f, device=device))
    return sd
