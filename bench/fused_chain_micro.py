"""Per-projection cost of the fused decode layer chain vs the plain (tuned) GEMMs, on the real
model's cold layer weights: python bench/fused_chain_micro.py [--model qwen3-0.6b]"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from aws_k8s_ansible_provisioner_amd import ops  # noqa: E402
from aws_k8s_ansible_provisioner_amd.models.config import get_config  # noqa: E402
from aws_k8s_ansible_provisioner_amd.models.transformer import DecoderLM  # noqa: E402
from aws_k8s_ansible_provisioner_amd.ops import gemm_tuner  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--model", default="qwen3-0.6b")
ap.add_argument("--m", default="64,128,256")
a = ap.parse_args()
ops.load_native(required=True)
m = DecoderLM(get_config(a.model), device="cuda")
Ms = [int(v) for v in a.m.split(",")]
gemm_tuner.tune_model(m, Ms)
gemm_tuner.tune_fused(m, Ms, verbose=True)
