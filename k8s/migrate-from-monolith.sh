#!/usr/bin/env bash
# Move an existing pre-split ("monolith": one Deployment `vgate` + Service `vgate`, optional HPA
# `vgate`, all labelled app=vgate) V-Gate install to the gateway / worker split.
#
# Why a script and not `kubectl apply -k`: apply never deletes objects that vanished from the
# manifests. The leftover monolith Deployment keeps its pods (and their GPUs), and the leftover
# Service `vgate` selects on app=vgate alone — which every pod of the split layout also carries,
# workers included — so traffic to the old Service name lands round-robin on the monolith, the
# new gateway AND the workers (which answer the public API with 404 by design). k8s/verify-migration.sh
# reproduces exactly that on kind and then runs this script.
#
#   k8s/migrate-from-monolith.sh --check            # exit 1 if monolith objects exist (no changes)
#   k8s/migrate-from-monolith.sh [--dry-run] [--overlay k8s/overlays/gpu] [--namespace vgate]
#
# Order: (1) find the monolith objects, (2) apply the split manifests and wait until the gateway
# is Ready with at least one worker admitted, (3) only then delete the monolith objects — the
# Service first (stops routing to the wrong pods), then the HPA (so it cannot scale the Deployment
# back up), then the Deployment; (4) verify nothing named `vgate` is left and the gateway serves.
set -euo pipefail

NS=vgate
OVERLAY=k8s/overlays/gpu
MODE=migrate
while [[ $# -gt 0 ]]; do
  case "$1" in
    --check) MODE=check; shift ;;
    --dry-run) MODE=dry; shift ;;
    --overlay) OVERLAY="$2"; shift 2 ;;
    --namespace) NS="$2"; shift 2 ;;
    migrate) shift ;;                    # accepted for compatibility with older callers
    k8s/*) OVERLAY="$1"; shift ;;
    *) echo "unknown argument: $1" >&2; exit 2 ;;
  esac
done

# the monolith's objects, in deletion order
ORPHANS=("service/vgate" "horizontalpodautoscaler/vgate" "deployment/vgate")

present=()
for o in "${ORPHANS[@]}"; do
  if kubectl -n "$NS" get "$o" >/dev/null 2>&1; then present+=("$o"); fi
done

if [[ "$MODE" == "check" ]]; then
  if (( ${#present[@]} )); then
    echo "monolith objects present in namespace $NS: ${present[*]}"
    # a Service selecting only app=vgate also matches the split layout's pods: say so
    sel=$(kubectl -n "$NS" get service/vgate -o jsonpath='{.spec.selector}' 2>/dev/null || true)
    [[ -n "$sel" ]] && echo "service/vgate selector: $sel (matches every app=vgate pod, gateway and workers included)"
    exit 1
  fi
  echo "no monolith objects in namespace $NS"
  exit 0
fi

echo "monolith objects: ${present[*]:-none}"
if [[ "$MODE" == "dry" ]]; then
  echo "[dry-run] would apply -k $OVERLAY, wait for vgate-gateway + vgate-worker, then delete: ${present[*]:-nothing}"
  kubectl apply -k "$OVERLAY" --dry-run=server >/dev/null
  echo "[dry-run] server-side dry run of the split manifests: OK"
  exit 0
fi

# (2) bring the split layout up first: the monolith keeps serving until its replacement is Ready
kubectl apply -k "$OVERLAY"
kubectl -n "$NS" rollout status deploy/vgate-gateway --timeout=600s
kubectl -n "$NS" rollout status statefulset/vgate-worker --timeout=1800s
ready=0
for _ in $(seq 1 90); do
  n=$(kubectl -n "$NS" exec deploy/vgate-gateway -c gateway -- python -c 'import json, urllib.request
s = json.load(urllib.request.urlopen("http://127.0.0.1:8000/stats", timeout=5))
print(sum(1 for w in s.get("workers", []) if w.get("healthy")))' 2>/dev/null || echo 0)
  if [[ "$n" -ge 1 ]]; then ready=1; break; fi
  sleep 2
done
if [[ "$ready" != 1 ]]; then
  echo "the new gateway never admitted a worker: leaving the monolith in place" >&2
  exit 1
fi

# (3) retire the monolith
for o in "${present[@]}"; do
  echo "deleting $o"
  kubectl -n "$NS" delete "$o" --wait=true
done

# (4) verify
left=()
for o in "${ORPHANS[@]}"; do kubectl -n "$NS" get "$o" >/dev/null 2>&1 && left+=("$o"); done
if (( ${#left[@]} )); then
  echo "still present after migration: ${left[*]}" >&2
  exit 1
fi
code=$(kubectl -n "$NS" exec deploy/vgate-gateway -c gateway -- python -c 'import urllib.request
print(urllib.request.urlopen("http://127.0.0.1:8000/health", timeout=5).status)' 2>/dev/null || echo 000)
[[ "$code" == "200" ]] || { echo "gateway /health answered $code after the migration" >&2; exit 1; }
echo "migration complete: split layout serving, no monolith objects left in $NS"
