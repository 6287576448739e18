"""llm-d-compatible installer for the MI355X serving stack.

Flag-compatible with the llm-d-deployer quickstart the reference drives
(llm-d-deploy.yaml:176-193): --values-file --namespace --storage-class --storage-size
--download-model, HF_TOKEN / KUBECONFIG from the environment.  It renders the manifests
under deploy/templates/ for a values preset (slim | pd | tp8 | moe | kind), writes them to
--output-dir and applies them with kubectl (skip with --dry-run).

    python -m aws_k8s_ansible_provisioner_amd.deploy.installer \
        --values-file deploy/values/slim.yaml --namespace llm-d \
        --storage-class local-path --storage-size 50Gi --download-model Qwen/Qwen3-0.6B
"""
from __future__ import annotations

import argparse
import json
import os
import shutil
import subprocess
import sys
from typing import Optional

import jinja2
import yaml

from ..utils import chat_template

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
TEMPLATES = os.path.join(ROOT, "deploy", "templates")
OTEL_TRACES_ENDPOINT = ("http://otel-metrics-collector-collector.observability.svc"
                        ".cluster.local:4318")
ORDER = ["base.yaml.j2", "engines.yaml.j2", "gateway.yaml.j2", "gpu-exporter.yaml.j2"]


def load_values(path: str) -> dict:
    with open(path) as f:
        v = yaml.safe_load(f)
    v.setdefault("engines", [{"role": "both", "replicas": 1, "gpusPerPod": 1,
                              "tensorParallel": 1}])
    v.setdefault("gateway", {"replicas": 1, "pdThresholdChars": 2048})
    # OTLP/HTTP traces -> the OTel collector DaemonSet of otel-observability-setup.yaml
    v.setdefault("tracing", {"endpoint": OTEL_TRACES_ENDPOINT})
    return v


def chat_configmaps(ns: str) -> list[str]:
    out = []
    for name in ("phi", "opt", "default"):
        doc = chat_template.configmap_yaml(name, chat_template.BUILTIN[name], ns)
        out.append(yaml.safe_dump(doc, sort_keys=False, width=4096))
    return out


def render(values: dict, ns: str = "llm-d", storage_class: str = "local-path",
           storage_size: str = "50Gi", download_model: Optional[str] = None,
           hf_token: Optional[str] = None, exporter_ns: str = "kube-amd-gpu",
           gateway_api: bool = False) -> dict[str, str]:
    """gateway_api: also emit a Gateway API `Gateway` + `HTTPRoute` named
    llm-d-inference-gateway in front of our gateway Service (tier 1 of the reference smoke
    test's address lookup, llm-d-test.yaml:16); the installer turns it on when the
    gateways.gateway.networking.k8s.io CRD exists in the cluster."""
    env = jinja2.Environment(loader=jinja2.FileSystemLoader(TEMPLATES), trim_blocks=True,
                             lstrip_blocks=True, undefined=jinja2.StrictUndefined)
    ctx = dict(v=values, ns=ns, storage_class=storage_class, storage_size=storage_size,
               download_model=download_model, hf_token=hf_token,
               chat_configmaps=chat_configmaps(ns), exporter_ns=exporter_ns,
               gateway_api=gateway_api)
    out = {}
    for name in ORDER:
        if name == "gpu-exporter.yaml.j2" and not values.get("gpuExporter", True):
            continue
        text = env.get_template(name).render(**ctx)
        docs = [d for d in yaml.safe_load_all(text) if d]  # validate: must parse
        out[name[:-3]] = yaml.safe_dump_all(docs, sort_keys=False, width=4096)
    return out


def kubectl(args: list[str], check: bool = True) -> subprocess.CompletedProcess:
    exe = shutil.which("kubectl")
    if exe is None:
        raise RuntimeError("kubectl not found on PATH")
    return subprocess.run([exe, *args], check=check, text=True, capture_output=True)


def main(argv=None) -> int:
    ap = argparse.ArgumentParser("akap-llmd-installer")
    ap.add_argument("--values-file", default=os.path.join(ROOT, "deploy", "values", "slim.yaml"))
    ap.add_argument("--namespace", default="llm-d")
    ap.add_argument("--storage-class", default="local-path")
    ap.add_argument("--storage-size", default="50Gi")
    ap.add_argument("--download-model", default=None)
    ap.add_argument("--output-dir", default="./akap-manifests")
    ap.add_argument("--dry-run", action="store_true")
    ap.add_argument("--uninstall", action="store_true")
    ap.add_argument("--wait-timeout", default="1800s")
    a = ap.parse_args(argv)
    values = load_values(a.values_file)
    gw_api = values.get("gatewayApi", "auto")
    if gw_api == "auto":
        gw_api = (not a.dry_run and shutil.which("kubectl") is not None and kubectl(
            ["get", "crd", "gateways.gateway.networking.k8s.io"], check=False).returncode == 0)
    manifests = render(values, a.namespace, a.storage_class, a.storage_size, a.download_model,
                       os.environ.get("HF_TOKEN") or None, gateway_api=bool(gw_api))
    os.makedirs(a.output_dir, exist_ok=True)
    paths = []
    for name, text in manifests.items():
        p = os.path.join(a.output_dir, name)
        with open(p, "w") as f:
            f.write(text)
        paths.append(p)
    print(json.dumps({"rendered": paths, "namespace": a.namespace, "model": values["model"]}))
    if a.dry_run:
        return 0
    if a.uninstall:
        for p in reversed(paths):
            kubectl(["delete", "--ignore-not-found", "-f", p], check=False)
        return 0
    for p in paths:
        r = kubectl(["apply", "-f", p])
        print(r.stdout, end="")
    r = kubectl(["wait", "--for=condition=available", "deployment", "--all", "-n",
                 a.namespace, f"--timeout={a.wait_timeout}"], check=False)
    print(r.stdout + r.stderr, end="")
    return r.returncode


if __name__ == "__main__":
    sys.exit(main())
