#!/usr/bin/env bash
# Live verification of the split deployment (gateway Deployment + worker StatefulSet behind a
# headless Service, DNS discovery) on a 3-node kind cluster with the CPU overlay (dry-run
# workers, 100 ms simulated generations). Validating manifests proves they parse; this proves
# they DEPLOY a working system: placement, per-pod DNS identity, traffic spread, failover under
# live load with zero unanswered probes, discovery-driven scale out / in / to zero and back.
#
# Every assertion prints [PASS]/[FAIL] through `claim`; the script runs to the end and exits
# with the number of failed claims (0 = all 26 held).
#
#   k8s/kind-verify.sh              # needs kind, kubectl, docker; KEEP=1 leaves the cluster up
#
# Behavioural parity target: reference k8s/kind-verify.sh (distinct nodes, per-pod DNS,
# traffic split, failover without unanswered probes, 503 at scale-to-zero, rejoin).
set -uo pipefail
cd "$(dirname "$0")/.."

NS=vgate
CLUSTER=vgate
IMAGE=vgate:0.3.2-cpu
KEY=change-me                      # k8s/base/secret.yaml api key (CPU overlay)
WORKER_DNS=vgate-worker.vgate.svc.cluster.local
FAILS=0
PASSES=0

step() { printf '\n== %s\n' "$*"; }
claim() {  # claim <0 = holds | anything else> <description>
  if [[ "$1" == "0" ]]; then
    echo "[PASS] $2"; PASSES=$((PASSES + 1))
  else
    echo "[FAIL] $2"; FAILS=$((FAILS + 1))
  fi
}
gw() {  # run a python snippet inside the gateway pod (stdlib only)
  kubectl -n "$NS" exec deploy/vgate-gateway -c gateway -- python -c "$1" 2>/dev/null
}
stats_py='import json, urllib.request
s = json.load(urllib.request.urlopen("http://127.0.0.1:8000/stats", timeout=5))
ws = s.get("workers", [])'
known_workers() { gw "$stats_py
print(len(ws))" || echo -1; }
healthy_workers() { gw "$stats_py
print(sum(1 for w in ws if w.get(\"healthy\")))" || echo -1; }
named_workers() { gw "$stats_py
print(sum(1 for w in ws if \"vgate-worker-\" in w[\"endpoint\"]))" || echo -1; }
wait_for() {  # wait_for <fn> <want> [timeout s]
  local fn="$1" want="$2" limit="${3:-150}" t=0 got
  while (( t < limit )); do
    got="$($fn)"
    [[ "$got" == "$want" ]] && { echo "$got"; return 0; }
    sleep 2; t=$((t + 2))
  done
  echo "$got"; return 1
}
ask() {  # one chat completion from inside the gateway pod; prints the HTTP status (000 = no answer)
  gw "import json, urllib.request, urllib.error
r = urllib.request.Request('http://127.0.0.1:8000/v1/chat/completions',
    data=json.dumps({'model': 'm', 'messages': [{'role': 'user', 'content': '''$1'''}], 'max_tokens': 4}).encode(),
    headers={'Content-Type': 'application/json', 'Authorization': 'Bearer $KEY'})
try:
    print(urllib.request.urlopen(r, timeout=30).status)
except urllib.error.HTTPError as e:
    print(e.code)
except Exception:
    print('000')" || echo 000
}
served_per_worker() {  # "<endpoint> <successes>" lines from the gateway's Prometheus counters
  gw 'import re, urllib.request
t = urllib.request.urlopen("http://127.0.0.1:8000/metrics", timeout=5).read().decode()
for m in re.finditer(r"vgate_worker_requests_total\{worker=\"([^\"]+)\",outcome=\"success\"\} ([0-9.e+]+)", t):
    print(m.group(1), int(float(m.group(2))))'
}
count_served() { served_per_worker | awk '$2 > 0' | wc -l; }
probe_burst() {  # probe_burst <n> <tag>: n sequential asks, prints one status per line
  gw "import json, urllib.request, urllib.error
for i in range($1):
    r = urllib.request.Request('http://127.0.0.1:8000/v1/chat/completions',
        data=json.dumps({'model': 'm', 'messages': [{'role': 'user', 'content': '$2 %d' % i}], 'max_tokens': 4}).encode(),
        headers={'Content-Type': 'application/json', 'Authorization': 'Bearer $KEY'})
    try:
        print(urllib.request.urlopen(r, timeout=30).status)
    except urllib.error.HTTPError as e:
        print(e.code)
    except Exception:
        print('000')"
}
scale() { kubectl -n "$NS" scale statefulset/vgate-worker --replicas="$1" >/dev/null; }

# ---------------------------------------------------------------------------------------
step "1. Cluster, image, manifests"
kind get clusters 2>/dev/null | grep -qx "$CLUSTER" || kind create cluster --name "$CLUSTER" --config k8s/kind-cluster.yaml
docker build --target cpu -t "$IMAGE" . >/dev/null && kind load docker-image "$IMAGE" --name "$CLUSTER" >/dev/null
python3 k8s/validate_manifests.py >/dev/null; claim "$?" "the manifests pass the offline validator"
kubectl apply -k k8s/overlays/cpu >/dev/null; claim "$?" "kubectl apply -k k8s/overlays/cpu succeeds"

step "2. Rollout"
kubectl -n "$NS" rollout status deploy/vgate-gateway --timeout=240s >/dev/null; claim "$?" "the gateway Deployment rolls out"
kubectl -n "$NS" rollout status statefulset/vgate-worker --timeout=240s >/dev/null; claim "$?" "the worker StatefulSet rolls out (2 replicas)"

step "3. Placement and identity"
worker_nodes=$(kubectl -n "$NS" get pods -l component=worker -o jsonpath='{range .items[*]}{.spec.nodeName}{"\n"}{end}' | sort -u | wc -l)
claim "$([[ "$worker_nodes" -eq 2 ]] && echo 0 || echo 1)" "the two workers run on different nodes (distinct nodes: $worker_nodes)"
resolved=$(gw "import socket
print(len({socket.gethostbyname('vgate-worker-%d.$WORKER_DNS' % i) for i in range(2)}))" || echo 0)
claim "$([[ "$resolved" -eq 2 ]] && echo 0 || echo 1)" "each worker has its own per-pod DNS name and address (distinct: $resolved)"
known=$(wait_for known_workers 2)
claim "$?" "the gateway discovered both workers through the headless Service (known: $known)"
byname=$(named_workers)
claim "$([[ "$byname" -eq 2 ]] && echo 0 || echo 1)" "workers are tracked by stable pod name, not address ($byname/2)"

step "4. Serving"
code=$(ask "hello from kind-verify")
claim "$([[ "$code" == "200" ]] && echo 0 || echo 1)" "a chat completion is served end to end through the gateway (HTTP $code)"
probe_burst 20 spread >/dev/null
used=$(count_served)
claim "$([[ "$used" -eq 2 ]] && echo 0 || echo 1)" "requests are spread over both workers (workers that served: $used)"
hz=$(gw 'import urllib.request
print(urllib.request.urlopen("http://127.0.0.1:8000/health", timeout=5).status)' || echo 000)
claim "$([[ "$hz" == "200" ]] && echo 0 || echo 1)" "/health answers 200 without credentials (exempt path)"

step "5. Failover under live traffic"
# probes run while vgate-worker-1 is deleted: every probe must be answered (no 000), none may
# see an empty pool (503) while a worker is up, and any other non-200 must be the documented
# non-retryable mid-request failure (500 from RemoteInferenceError), never a hang
probe_burst 60 failover > /tmp/vgate_failover_codes.txt &
PROBES=$!
sleep 1
kubectl -n "$NS" delete pod vgate-worker-1 --wait=false >/dev/null
wait "$PROBES"
p000=$(grep -c '^000$' /tmp/vgate_failover_codes.txt)
p503=$(grep -c '^503$' /tmp/vgate_failover_codes.txt)
pother=$(grep -vcE '^(200|000|503|500)$' /tmp/vgate_failover_codes.txt)
claim "$([[ "$p000" -eq 0 ]] && echo 0 || echo 1)" "no probe went unanswered during the worker kill (000: $p000 of 60)"
claim "$([[ "$p503" -eq 0 ]] && echo 0 || echo 1)" "the pool never reported itself empty while a worker was up (503: $p503)"
claim "$([[ "$pother" -eq 0 ]] && echo 0 || echo 1)" "every non-200 is the non-retryable mid-request class (unexpected codes: $pother)"
serving=$(healthy_workers)
claim "$([[ "$serving" -ge 1 ]] && echo 0 || echo 1)" "the survivor kept serving (healthy workers: $serving)"
back=$(wait_for healthy_workers 2 180)
claim "$?" "the recreated pod (same stable name) is re-admitted (healthy: $back)"

step "6. Scale out / in through discovery (no gateway edit)"
scale 3
kubectl -n "$NS" rollout status statefulset/vgate-worker --timeout=240s >/dev/null
k3=$(wait_for known_workers 3)
claim "$?" "scaling out to 3 is discovered without touching the gateway (known: $k3)"
probe_burst 30 three >/dev/null
s3=$(served_per_worker | grep -c 'vgate-worker-2')
claim "$([[ "$s3" -eq 1 ]] && echo 0 || echo 1)" "the new third worker serves traffic"
scale 2
k2=$(wait_for known_workers 2)
claim "$?" "a removed worker stops being tracked rather than probed forever (known: $k2)"

step "7. Scale to zero and back"
scale 0
k0=$(wait_for known_workers 0 240)
claim "$?" "scaling to zero empties the registry after the confirmation streak (known: $k0)"
zero=$(ask "empty pool probe")
claim "$([[ "$zero" == "503" ]] && echo 0 || echo 1)" "an empty pool answers 503 instead of hanging (HTTP $zero)"
before=$(served_per_worker | awk '{s+=$2} END {print s+0}')
scale 2
kubectl -n "$NS" rollout status statefulset/vgate-worker --timeout=240s >/dev/null
kr=$(wait_for healthy_workers 2 240)
claim "$?" "the emptied pool repopulates and both workers are admitted (healthy: $kr)"
again=$(ask "after the pool came back")
claim "$([[ "$again" == "200" ]] && echo 0 || echo 1)" "the gateway serves again after the pool comes back (HTTP $again)"
probe_burst 10 rejoin >/dev/null
after=$(served_per_worker | awk '{s+=$2} END {print s+0}')
claim "$(python3 -c "print(0 if $after > $before else 1)")" "returned workers serve new requests ($before -> $after successes)"

step "8. Observability"
metrics_ok=$(gw 'import urllib.request
t = urllib.request.urlopen("http://127.0.0.1:8000/metrics", timeout=5).read().decode()
print(0 if "vgate_worker_healthy" in t and "vgate_requests_total" in t else 1)' || echo 1)
claim "$metrics_ok" "/metrics exports per-worker health and request counters"
hpa=$(kubectl -n "$NS" get hpa vgate-gateway -o name 2>/dev/null | wc -l)
claim "$([[ "$hpa" -eq 1 ]] && echo 0 || echo 1)" "the gateway HorizontalPodAutoscaler is installed"

printf '\n%d claims held, %d failed\n' "$PASSES" "$FAILS"
[[ "${KEEP:-0}" == "1" ]] || kind delete cluster --name "$CLUSTER" >/dev/null 2>&1
exit "$FAILS"
