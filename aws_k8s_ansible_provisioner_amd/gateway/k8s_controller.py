"""Minimal Gateway API controller for GatewayClass ``akap`` (runs inside the gateway pod).

The reference's smoke test looks the gateway up in three tiers, the first being
``Gateway.status.addresses[0].value`` (/root/reference/llm-d-test.yaml:14-26).  llm-d's
quickstart installs a Gateway API implementation whose controller fills that status; ours
is this reconcile loop: the gateway process IS the data plane, so "programming" a Gateway of
our class means publishing the ClusterIP of the Service in front of it.

Every ``interval`` seconds (level-triggered, idempotent, safe with several gateway
replicas reconciling the same objects):
  * GatewayClass whose ``spec.controllerName`` is ours -> status Accepted=True;
  * every Gateway of that class in our namespace -> status.addresses = [IPAddress of the
    Service named like the Gateway (the data-plane Service)], Accepted/Programmed
    conditions, and per-listener status with the attached-route count;
  * every HTTPRoute whose parentRef names such a Gateway -> status.parents Accepted +
    ResolvedRefs for our controller.
Talks to the API server over its REST API with the pod's service-account token (the
``kubernetes`` client package is not a dependency); in tests, against a fake server.
"""
from __future__ import annotations

import asyncio
import json
import os
import ssl
import time
from typing import Optional

import aiohttp

CONTROLLER_NAME = "akap.ai/inference-gateway-controller"
GW_API = "/apis/gateway.networking.k8s.io/v1"
SA_DIR = "/var/run/secrets/kubernetes.io/serviceaccount"


def _cond(ctype: str, reason: str, generation: int, msg: str = "") -> dict:
    return {"type": ctype, "status": "True", "reason": reason, "message": msg,
            "observedGeneration": generation,
            "lastTransitionTime": time.strftime("%Y-%m-%dT%H:%M:%SZ", time.gmtime())}


def _same_conditions(old: list, new: list) -> bool:
    """Ignore lastTransitionTime: only a real change is written back."""
    strip = lambda cs: sorted((c.get("type"), c.get("status"), c.get("reason"),  # noqa: E731
                               c.get("observedGeneration")) for c in cs or [])
    return strip(old) == strip(new)


class GatewayController:
    def __init__(self, namespace: str, api: Optional[str] = None, token: Optional[str] = None,
                 ca_file: Optional[str] = None, class_name: str = "akap",
                 interval: float = 10.0):
        if api is None:
            host = os.environ.get("KUBERNETES_SERVICE_HOST", "kubernetes.default.svc")
            port = os.environ.get("KUBERNETES_SERVICE_PORT", "443")
            api = f"https://{host}:{port}"
        self.api = api.rstrip("/")
        if token is None and os.path.exists(os.path.join(SA_DIR, "token")):
            token = open(os.path.join(SA_DIR, "token")).read().strip()
        self.token = token
        self.ca_file = ca_file if ca_file is not None else (
            os.path.join(SA_DIR, "ca.crt") if os.path.exists(os.path.join(SA_DIR, "ca.crt"))
            else None)
        self.ns = namespace
        self.class_name = class_name
        self.interval = interval
        self.reconciles = 0
        self.errors = 0
        self.last_error: Optional[str] = None

    # ---------------------------------------------------------------- REST helpers
    def _headers(self, patch: bool = False) -> dict:
        h = {"Accept": "application/json"}
        if self.token:
            h["Authorization"] = f"Bearer {self.token}"
        if patch:
            h["Content-Type"] = "application/merge-patch+json"
        return h

    def _ssl(self):
        """TLS context for the API server.  Fails closed: a bearer token is never sent over a
        connection whose certificate is not verified (no service-account ca.crt -> the system
        trust store, never verification off)."""
        if not self.api.startswith("https"):
            host = self.api.split("://", 1)[-1].split("/", 1)[0].rsplit(":", 1)[0]
            if self.token and host not in ("127.0.0.1", "localhost", "[::1]"):
                # plain HTTP only to a loopback endpoint (kubectl proxy, tests)
                raise RuntimeError("refusing to send the service-account token over plain HTTP")
            return None
        return ssl.create_default_context(cafile=self.ca_file)

    async def _get(self, s: aiohttp.ClientSession, path: str) -> Optional[dict]:
        async with s.get(self.api + path, headers=self._headers(), ssl=self._ssl()) as r:
            if r.status == 404:
                return None
            r.raise_for_status()
            return await r.json()

    async def _patch_status(self, s: aiohttp.ClientSession, path: str, status: dict) -> None:
        async with s.patch(self.api + path + "/status", data=json.dumps({"status": status}),
                           headers=self._headers(patch=True), ssl=self._ssl()) as r:
            r.raise_for_status()

    # ---------------------------------------------------------------- reconcile
    async def reconcile(self, s: aiohttp.ClientSession) -> dict:
        """One level-triggered pass; returns what it programmed (for tests / logs)."""
        done = {"gatewayclass": False, "gateways": {}, "routes": []}
        gc = await self._get(s, f"{GW_API}/gatewayclasses/{self.class_name}")
        if gc is None or gc.get("spec", {}).get("controllerName") != CONTROLLER_NAME:
            return done  # another implementation owns this class (or it does not exist)
        gen = gc["metadata"].get("generation", 1)
        conds = [_cond("Accepted", "Accepted", gen, "akap inference gateway")]
        if not _same_conditions(gc.get("status", {}).get("conditions"), conds):
            await self._patch_status(s, f"{GW_API}/gatewayclasses/{self.class_name}",
                                     {"conditions": conds})
        done["gatewayclass"] = True
        gws = (await self._get(s, f"{GW_API}/namespaces/{self.ns}/gateways")) or {"items": []}
        ours = [g for g in gws["items"] if g["spec"].get("gatewayClassName") == self.class_name]
        routes = (await self._get(s, f"{GW_API}/namespaces/{self.ns}/httproutes")) or \
            {"items": []}
        attached: dict = {}
        for rt in routes["items"]:
            parents = [p for p in rt["spec"].get("parentRefs", [])
                       if p.get("name") in {g["metadata"]["name"] for g in ours}
                       and p.get("namespace", self.ns) == self.ns]
            for p in parents:
                attached[p["name"]] = attached.get(p["name"], 0) + 1
            if parents:
                rgen = rt["metadata"].get("generation", 1)
                st = {"parents": [{"parentRef": {"name": p["name"], "namespace": self.ns,
                                                 "group": "gateway.networking.k8s.io",
                                                 "kind": "Gateway"},
                                   "controllerName": CONTROLLER_NAME,
                                   "conditions": [_cond("Accepted", "Accepted", rgen),
                                                  _cond("ResolvedRefs", "ResolvedRefs", rgen)]}
                                  for p in parents]}
                await self._patch_status(
                    s, f"{GW_API}/namespaces/{self.ns}/httproutes/{rt['metadata']['name']}", st)
                done["routes"].append(rt["metadata"]["name"])
        for g in ours:
            name = g["metadata"]["name"]
            svc = await self._get(s, f"/api/v1/namespaces/{self.ns}/services/{name}")
            ip = (svc or {}).get("spec", {}).get("clusterIP")
            if not ip or ip == "None":
                continue  # data-plane Service not there yet: next pass
            ggen = g["metadata"].get("generation", 1)
            st = {"addresses": [{"type": "IPAddress", "value": ip}],
                  "conditions": [_cond("Accepted", "Accepted", ggen),
                                 _cond("Programmed", "Programmed", ggen,
                                       f"served by Service {name}")],
                  "listeners": [{"name": ln["name"], "attachedRoutes": attached.get(name, 0),
                                 "supportedKinds": [{"group": "gateway.networking.k8s.io",
                                                     "kind": "HTTPRoute"}],
                                 "conditions": [_cond("Accepted", "Accepted", ggen),
                                                _cond("Programmed", "Programmed", ggen),
                                                _cond("ResolvedRefs", "ResolvedRefs", ggen)]}
                                for ln in g["spec"].get("listeners", [])]}
            old = g.get("status", {})
            if old.get("addresses") != st["addresses"] or not _same_conditions(
                    old.get("conditions"), st["conditions"]):
                await self._patch_status(s, f"{GW_API}/namespaces/{self.ns}/gateways/{name}", st)
            done["gateways"][name] = ip
        self.reconciles += 1
        return done

    async def run(self) -> None:
        async with aiohttp.ClientSession(timeout=aiohttp.ClientTimeout(total=15)) as s:
            while True:
                try:
                    await self.reconcile(s)
                    self.last_error = None
                except (aiohttp.ClientError, asyncio.TimeoutError, OSError, KeyError,
                        ValueError) as e:  # API server unreachable / CRDs absent: retry later
                    self.errors += 1
                    self.last_error = f"{type(e).__name__}: {e}"
                await asyncio.sleep(self.interval)


def in_cluster() -> bool:
    return bool(os.environ.get("KUBERNETES_SERVICE_HOST")) and \
        os.path.exists(os.path.join(SA_DIR, "token"))
