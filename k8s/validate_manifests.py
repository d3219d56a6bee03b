#!/usr/bin/env python3
"""Static invariants of the V-Gate Kubernetes manifests (no cluster needed).

Renders base + each overlay with a small built-in strategic merge (containers and env
merged by name, maps merged recursively — enough for the patches in k8s/overlays) and
checks the split-deployment contract:

  1. the gateway holds no model and no GPU (no accelerator resources, no weights path);
  2. the worker Service is headless and publishes not-ready addresses;
  3. the gateway Service selects only gateway pods;
  4. gateway DNS discovery targets the worker Service;
  5. no unresolved ``$(VAR)`` references in env values;
  6. every image is pinned (no ``:latest``, tag present) with an explicit pull policy;
  7. overlays agree with the base on immutable fields (selectors, serviceName,
     volumeClaimTemplates);
  8. the GPU overlay requests ``amd.com/gpu`` for workers and uses the ROCm image.

Exit status 0 = all invariants hold; otherwise every violation is printed.

    python k8s/validate_manifests.py
"""
from __future__ import annotations

import copy
import sys
from pathlib import Path

import yaml

ROOT = Path(__file__).resolve().parent
ACCEL = ("amd.com/gpu", "nvidia.com/gpu")


def load_docs(path: Path) -> list[dict]:
    return [d for d in yaml.safe_load_all(path.read_text()) if d]


def kustomize(dir_: Path) -> list[dict]:
    k = yaml.safe_load((dir_ / "kustomization.yaml").read_text())
    docs: list[dict] = []
    for r in k.get("resources", []):
        p = dir_ / r
        docs += kustomize(p) if p.is_dir() else load_docs(p)
    for patch in k.get("patches", []):
        for pd in load_docs(dir_ / patch["path"]):
            for d in docs:
                if d["kind"] == pd["kind"] and d["metadata"]["name"] == pd["metadata"]["name"]:
                    merge(d, pd)
    ns = k.get("namespace")
    if ns:
        for d in docs:
            if d["kind"] != "Namespace":
                d["metadata"]["namespace"] = ns
    return docs


def merge(base, patch):
    """Strategic-merge subset: dicts recursively; lists of named dicts by 'name'."""
    for key, val in patch.items():
        if isinstance(val, dict) and isinstance(base.get(key), dict):
            merge(base[key], val)
        elif isinstance(val, list) and isinstance(base.get(key), list) and val and all(
                isinstance(x, dict) and "name" in x for x in val):
            by = {x.get("name"): x for x in base[key] if isinstance(x, dict)}
            for x in val:
                if x["name"] in by:
                    merge(by[x["name"]], x)
                else:
                    base[key].append(copy.deepcopy(x))
        else:
            base[key] = copy.deepcopy(val)
    return base


def find(docs, kind, name):
    for d in docs:
        if d["kind"] == kind and d["metadata"]["name"] == name:
            return d
    return None


def containers(d):
    return d["spec"]["template"]["spec"].get("containers", [])


def env_of(c):
    return {e["name"]: e.get("value") for e in c.get("env", [])}


def check(docs: list[dict], label: str, base_docs: list[dict] | None, errs: list[str]) -> None:
    def err(msg):
        errs.append(f"[{label}] {msg}")

    gw = find(docs, "Deployment", "vgate-gateway")
    wk = find(docs, "StatefulSet", "vgate-worker")
    wsvc = find(docs, "Service", "vgate-worker")
    gsvc = find(docs, "Service", "vgate-gateway")
    for name, obj in (("gateway Deployment", gw), ("worker StatefulSet", wk), ("worker Service", wsvc),
                      ("gateway Service", gsvc)):
        if obj is None:
            err(f"missing {name}")
    if None in (gw, wk, wsvc, gsvc):
        return
    # 1. gateway: no accelerators, no model weights
    for c in containers(gw):
        res = c.get("resources", {})
        for part in ("requests", "limits"):
            for acc in ACCEL:
                if acc in (res.get(part) or {}):
                    err(f"gateway container {c['name']} requests {acc}")
        env = env_of(c)
        if env.get("VGATE_MODEL__WEIGHTS_PATH"):
            err("gateway must not load model weights")
        if env.get("VGATE_ROLE") != "gateway":
            err("gateway container must set VGATE_ROLE=gateway")
    # 2. headless worker service
    if wsvc["spec"].get("clusterIP") != "None":
        err("worker Service must be headless (clusterIP: None)")
    if not wsvc["spec"].get("publishNotReadyAddresses"):
        err("worker Service must publishNotReadyAddresses (the gateway health-checks admission itself)")
    # 3. gateway service selects only gateway pods
    sel = gsvc["spec"].get("selector", {})
    if sel.get("component") != "gateway":
        err(f"gateway Service selector {sel} must pin component=gateway")
    # 4. discovery targets the worker service
    dns = None
    for c in containers(gw):
        dns = env_of(c).get("VGATE_WORKER__DISCOVERY__DNS_NAME") or dns
    ns = wsvc["metadata"].get("namespace", "default")
    if not dns or not dns.startswith(f"{wsvc['metadata']['name']}.{ns}"):
        err(f"gateway discovery DNS {dns!r} must target the worker Service {wsvc['metadata']['name']}.{ns}")
    if wk["spec"].get("serviceName") != wsvc["metadata"]["name"]:
        err("worker StatefulSet serviceName must be the headless worker Service")
    for d in docs:
        if d["kind"] not in ("Deployment", "StatefulSet"):
            continue
        for c in containers(d):
            # 5. unresolved references
            for e in c.get("env", []):
                v = e.get("value")
                if isinstance(v, str) and "$(" in v:
                    err(f"{d['metadata']['name']}/{c['name']}: unresolved reference in {e['name']}={v}")
            # 6. pinned images
            img = c.get("image", "")
            tag = img.rsplit(":", 1)[-1] if ":" in img.rsplit("/", 1)[-1] else ""
            if not tag or tag == "latest":
                err(f"{d['metadata']['name']}/{c['name']}: image {img!r} must be pinned")
            if "imagePullPolicy" not in c:
                err(f"{d['metadata']['name']}/{c['name']}: explicit imagePullPolicy required")
    # 7. immutable fields vs base
    if base_docs is not None:
        for kind, name, paths in (("StatefulSet", "vgate-worker", (("spec", "selector"), ("spec", "serviceName"),
                                                                   ("spec", "volumeClaimTemplates"))),
                                  ("Deployment", "vgate-gateway", (("spec", "selector"),))):
            a, b = find(docs, kind, name), find(base_docs, kind, name)
            for path in paths:
                va, vb = a, b
                for p in path:
                    va, vb = (va or {}).get(p), (vb or {}).get(p)
                if va != vb:
                    err(f"{kind}/{name}: immutable field {'.'.join(path)} differs from base")


def main() -> int:
    errs: list[str] = []
    base = kustomize(ROOT / "base")
    check(base, "base", None, errs)
    for ov in sorted((ROOT / "overlays").iterdir()):
        if (ov / "kustomization.yaml").exists():
            docs = kustomize(ov)
            check(docs, ov.name, base, errs)
            if ov.name == "gpu":  # 8.
                wk = find(docs, "StatefulSet", "vgate-worker")
                for c in containers(wk):
                    req = (c.get("resources") or {}).get("limits") or {}
                    if "amd.com/gpu" not in req:
                        errs.append("[gpu] worker must request amd.com/gpu")
                    if "rocm" not in c.get("image", ""):
                        errs.append("[gpu] worker must use the ROCm image")
    for e in errs:
        print("FAIL", e)
    if not errs:
        print("OK: all manifest invariants hold (base + overlays)")
    return 1 if errs else 0


if __name__ == "__main__":
    sys.exit(main())
