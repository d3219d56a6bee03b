#!/usr/bin/env bash
# Reproduce the migration hazard on kind and verify migrate-from-monolith.sh fixes it:
# a leftover monolith Service would split traffic with the new gateway.
set -euo pipefail
NS=vgate
kubectl create namespace $NS --dry-run=client -o yaml | kubectl apply -f -
kubectl -n $NS create deployment vgate --image=vgate:0.3.2-cpu --dry-run=client -o yaml | kubectl apply -f -
kubectl -n $NS expose deployment vgate --port 8000 --dry-run=client -o yaml | kubectl apply -f -
if k8s/migrate-from-monolith.sh --check; then echo "[FAIL] hazard not reproduced"; exit 1; fi
echo "[PASS] hazard reproduced (monolith objects present)"
k8s/migrate-from-monolith.sh migrate k8s/overlays/cpu
k8s/migrate-from-monolith.sh --check && echo "[PASS] migration removed the monolith"
