#!/usr/bin/env bash
# Migrate a pre-split (monolith) V-Gate install to the gateway/worker split. The monolith
# objects share names with nothing in the split layout but would keep serving traffic and
# holding GPUs; delete them BEFORE applying the split manifests.
#   k8s/migrate-from-monolith.sh [--check] [overlay]
set -euo pipefail
NS=vgate
OVERLAY="${2:-k8s/overlays/gpu}"
ORPHANS=("deployment/vgate" "service/vgate" "horizontalpodautoscaler/vgate")
found=()
for o in "${ORPHANS[@]}"; do
  kubectl -n $NS get "$o" >/dev/null 2>&1 && found+=("$o")
done
if [ "${1:-}" = "--check" ]; then
  if [ ${#found[@]} -gt 0 ]; then echo "monolith objects present: ${found[*]}"; exit 1; fi
  echo "no monolith objects"; exit 0
fi
for o in "${found[@]}"; do kubectl -n $NS delete "$o" --wait=true; done
kubectl apply -k "$OVERLAY"
kubectl -n $NS rollout status deploy/vgate-gateway --timeout=300s
kubectl -n $NS rollout status statefulset/vgate-worker --timeout=900s
