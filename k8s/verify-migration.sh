#!/usr/bin/env bash
# Reproduce the upgrade hazard on kind and show k8s/migrate-from-monolith.sh clearing it, with
# live traffic as the evidence (label arithmetic alone would only suggest it):
#
#   phase 1  deploy a pre-split monolith (Deployment `vgate` + Service `vgate`, selector app=vgate)
#            and confirm it serves through the `vgate` Service;
#   phase 2  upgrade the UNSAFE way, `kubectl apply -k` of the split manifests alone, then send
#            traffic to the old Service name and count which kind of pod answered: the monolith
#            is still there and the leftover Service spreads requests over monolith, gateway AND
#            workers (a worker answers the public API with 404);
#   phase 3  run the migration script and confirm only the split objects remain, the old
#            Service name no longer routes anywhere, and the new gateway serves.
# Every claim prints [PASS]/[FAIL]; the exit status is the number of failed claims.
#
#   k8s/verify-migration.sh        # needs kind, kubectl, docker (cluster from k8s/kind-cluster.yaml)
set -uo pipefail
cd "$(dirname "$0")/.."
NS=vgate
CLUSTER=vgate
IMAGE=vgate:0.3.2-cpu
FAILS=0
claim() { if [[ "$1" == "0" ]]; then echo "[PASS] $2"; else echo "[FAIL] $2"; FAILS=$((FAILS + 1)); fi; }

kind get clusters 2>/dev/null | grep -qx "$CLUSTER" || kind create cluster --name "$CLUSTER" --config k8s/kind-cluster.yaml
docker build --target cpu -t "$IMAGE" . >/dev/null && kind load docker-image "$IMAGE" --name "$CLUSTER" >/dev/null
kubectl delete namespace "$NS" --ignore-not-found --wait=true >/dev/null
kubectl create namespace "$NS" >/dev/null

# ---- phase 1: the pre-split monolith (what an older release deployed) -------------------------
kubectl -n "$NS" apply -f - >/dev/null <<'YAML'
apiVersion: apps/v1
kind: Deployment
metadata: {name: vgate, labels: {app: vgate}}
spec:
  replicas: 1
  selector: {matchLabels: {app: vgate}}
  template:
    metadata: {labels: {app: vgate}}
    spec:
      containers:
        - name: vgate
          image: vgate:0.3.2-cpu
          imagePullPolicy: IfNotPresent
          env: [{name: VGATE_DRY_RUN, value: "true"}, {name: VGATE_ROLE, value: gateway}]
          ports: [{containerPort: 8000}]
          readinessProbe: {httpGet: {path: /health, port: 8000}, periodSeconds: 2}
---
apiVersion: v1
kind: Service
metadata: {name: vgate, labels: {app: vgate}}
spec:
  selector: {app: vgate}
  ports: [{port: 8000, targetPort: 8000}]
YAML
kubectl -n "$NS" rollout status deploy/vgate --timeout=180s >/dev/null
claim "$?" "phase 1: the monolith rolls out"
# a throwaway client pod inside the cluster
kubectl -n "$NS" run probe --image="$IMAGE" --image-pull-policy=IfNotPresent --restart=Never \
  --command -- sleep 3600 >/dev/null
kubectl -n "$NS" wait --for=condition=Ready pod/probe --timeout=120s >/dev/null
through_old_service() {  # n requests to the OLD service name; prints one HTTP status per line
  kubectl -n "$NS" exec probe -- python -c "import json, urllib.request, urllib.error
for i in range($1):
    r = urllib.request.Request('http://vgate.$NS.svc.cluster.local:8000/v1/chat/completions',
        data=json.dumps({'model': 'm', 'messages': [{'role': 'user', 'content': 'm %d' % i}], 'max_tokens': 2}).encode(),
        headers={'Content-Type': 'application/json', 'Authorization': 'Bearer change-me'})
    try:
        print(urllib.request.urlopen(r, timeout=20).status)
    except urllib.error.HTTPError as e:
        print(e.code)
    except Exception:
        print('000')" 2>/dev/null
}
ok1=$(through_old_service 10 | grep -c '^200$')
claim "$([[ "$ok1" -eq 10 ]] && echo 0 || echo 1)" "phase 1: the monolith serves through Service vgate ($ok1/10)"

# ---- phase 2: the unsafe upgrade ---------------------------------------------------------------
kubectl apply -k k8s/overlays/cpu >/dev/null
kubectl -n "$NS" rollout status deploy/vgate-gateway --timeout=240s >/dev/null
kubectl -n "$NS" rollout status statefulset/vgate-worker --timeout=240s >/dev/null
still=$(kubectl -n "$NS" get deploy/vgate svc/vgate -o name 2>/dev/null | wc -l)
claim "$([[ "$still" -eq 2 ]] && echo 0 || echo 1)" "phase 2: apply alone leaves the monolith Deployment and Service behind ($still/2)"
eps=$(kubectl -n "$NS" get endpoints vgate -o jsonpath='{range .subsets[*].addresses[*]}{.targetRef.name}{"\n"}{end}')
workers_behind=$(echo "$eps" | grep -c '^vgate-worker-')
gw_behind=$(echo "$eps" | grep -c '^vgate-gateway-')
claim "$([[ "$workers_behind" -ge 1 && "$gw_behind" -ge 1 ]] && echo 0 || echo 1)" \
  "phase 2: the leftover Service now also selects the new gateway and the workers (gateway pods: $gw_behind, workers: $workers_behind)"
codes=$(through_old_service 40)
# a worker refuses the public API: 404 (gateway-only route), or 401 first if its internal key
# differs from the client's
n404=$(echo "$codes" | grep -cE '^(404|401)$')
claim "$([[ "$n404" -ge 1 ]] && echo 0 || echo 1)" \
  "phase 2: live traffic to the old name lands on workers, which refuse the public API ($n404/40 refused)"
k8s/migrate-from-monolith.sh --check --namespace "$NS" >/dev/null
claim "$([[ $? -eq 1 ]] && echo 0 || echo 1)" "phase 2: the migration pre-check detects the monolith"

# ---- phase 3: the migration --------------------------------------------------------------------
k8s/migrate-from-monolith.sh --overlay k8s/overlays/cpu --namespace "$NS"
claim "$?" "phase 3: the migration script completes"
k8s/migrate-from-monolith.sh --check --namespace "$NS" >/dev/null
claim "$?" "phase 3: no monolith objects remain"
left=$(kubectl -n "$NS" get deploy,svc -o name | grep -cE '/vgate$')
claim "$([[ "$left" -eq 0 ]] && echo 0 || echo 1)" "phase 3: nothing named vgate is left ($left)"
gone=$(through_old_service 3 | grep -c '^000$')
claim "$([[ "$gone" -eq 3 ]] && echo 0 || echo 1)" "phase 3: the old Service name routes nowhere ($gone/3 unanswered)"
new_ok=$(kubectl -n "$NS" exec probe -- python -c "import json, urllib.request
r = urllib.request.Request('http://vgate-gateway.$NS.svc.cluster.local:8000/v1/chat/completions',
    data=json.dumps({'model': 'm', 'messages': [{'role': 'user', 'content': 'after'}], 'max_tokens': 2}).encode(),
    headers={'Content-Type': 'application/json', 'Authorization': 'Bearer change-me'})
print(urllib.request.urlopen(r, timeout=20).status)" 2>/dev/null || echo 000)
claim "$([[ "$new_ok" == "200" ]] && echo 0 || echo 1)" "phase 3: the split gateway serves (HTTP $new_ok)"

kubectl -n "$NS" delete pod probe --wait=false >/dev/null 2>&1
echo "failed claims: $FAILS"
exit "$FAILS"
