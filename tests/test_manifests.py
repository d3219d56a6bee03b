"""k8s manifest invariants (k8s/validate_manifests.py): the shipped base + overlays pass,
and each invariant actually fires on a violating manifest."""
import copy
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1] / "k8s"))

import validate_manifests as vm  # noqa: E402


def _base():
    return vm.kustomize(vm.ROOT / "base")


def test_shipped_manifests_pass(capsys):
    assert vm.main() == 0
    assert "OK" in capsys.readouterr().out


def test_gpu_overlay_requests_amd_gpu():
    docs = vm.kustomize(vm.ROOT / "overlays" / "gpu")
    wk = vm.find(docs, "StatefulSet", "vgate-worker")
    c = vm.containers(wk)[0]
    assert c["resources"]["limits"]["amd.com/gpu"] == 1
    assert c["image"].endswith("rocm")
    gw = vm.find(docs, "Deployment", "vgate-gateway")
    assert "amd.com/gpu" not in str(gw)


def _violations(mutate):
    docs = copy.deepcopy(_base())
    mutate(docs)
    errs = []
    vm.check(docs, "t", _base(), errs)
    return errs


def test_invariants_fire():
    def gpu_on_gateway(d):
        vm.containers(vm.find(d, "Deployment", "vgate-gateway"))[0]["resources"]["limits"]["amd.com/gpu"] = 1
    assert any("gateway container" in e for e in _violations(gpu_on_gateway))

    def not_headless(d):
        vm.find(d, "Service", "vgate-worker")["spec"]["clusterIP"] = "10.0.0.1"
    assert any("headless" in e for e in _violations(not_headless))

    def latest(d):
        vm.containers(vm.find(d, "StatefulSet", "vgate-worker"))[0]["image"] = "vgate:latest"
    assert any("pinned" in e for e in _violations(latest))

    def unresolved(d):
        vm.containers(vm.find(d, "Deployment", "vgate-gateway"))[0]["env"].append({"name": "X", "value": "$(FOO)"})
    assert any("unresolved" in e for e in _violations(unresolved))

    def wrong_dns(d):
        for e in vm.containers(vm.find(d, "Deployment", "vgate-gateway"))[0]["env"]:
            if e["name"] == "VGATE_WORKER__DISCOVERY__DNS_NAME":
                e["value"] = "elsewhere.svc"
    assert any("discovery" in e for e in _violations(wrong_dns))

    def immutable(d):
        vm.find(d, "StatefulSet", "vgate-worker")["spec"]["serviceName"] = "other"
    assert any("immutable" in e or "serviceName" in e for e in _violations(immutable))
