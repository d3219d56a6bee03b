#!/usr/bin/env bash
# Live-cluster verification of the split deployment on a 3-node kind cluster (CPU overlay,
# dry-run workers): deploy, serve traffic, kill a worker under load, scale 1->3->2->0->2.
# Every claim prints [PASS]/[FAIL]; the script exits non-zero if any claim failed.
#   k8s/kind-verify.sh            # needs: kind, kubectl, docker
set -uo pipefail
cd "$(dirname "$0")/.."
NS=vgate
FAILS=0
claim() {  # claim "<description>" <command...>
  local desc="$1"; shift
  if "$@" >/dev/null 2>&1; then echo "[PASS] $desc"; else echo "[FAIL] $desc"; FAILS=$((FAILS + 1)); fi
}
wait_ready_workers() {  # wait until the gateway reports N healthy workers in /stats
  local want="$1" t=0
  while [ $t -lt 120 ]; do
    n=$(kubectl -n $NS exec deploy/vgate-gateway -- python -c \
      "import json,urllib.request;s=json.load(urllib.request.urlopen('http://127.0.0.1:8000/stats'));print(sum(w.get('healthy',False) for w in s.get('workers',[])))" 2>/dev/null || echo -1)
    [ "$n" = "$want" ] && return 0
    sleep 2; t=$((t + 2))
  done
  return 1
}
chat() {
  kubectl -n $NS exec deploy/vgate-gateway -- python -c \
    "import json,urllib.request;r=urllib.request.Request('http://127.0.0.1:8000/v1/chat/completions',data=json.dumps({'model':'m','messages':[{'role':'user','content':'hi $1'}],'max_tokens':4}).encode(),headers={'Content-Type':'application/json','Authorization':'Bearer change-me'});print(urllib.request.urlopen(r).status)"
}

kind get clusters | grep -qx vgate || kind create cluster --config k8s/kind-cluster.yaml
docker build --target cpu -t vgate:0.3.2-cpu . >/dev/null
kind load docker-image vgate:0.3.2-cpu --name vgate
python k8s/validate_manifests.py
kubectl apply -k k8s/overlays/cpu
claim "gateway rolls out" kubectl -n $NS rollout status deploy/vgate-gateway --timeout=180s
claim "workers roll out" kubectl -n $NS rollout status statefulset/vgate-worker --timeout=180s
claim "gateway admits 2 workers" wait_ready_workers 2
claim "chat completion through the gateway" chat 1
# kill a worker under traffic: requests keep succeeding on the survivor
( for i in $(seq 1 30); do chat "load$i" || true; done ) &
LOAD=$!
kubectl -n $NS delete pod vgate-worker-0 --wait=false
wait $LOAD
claim "traffic survives a worker kill" chat 2
claim "killed worker re-admitted" wait_ready_workers 2
for n in 1 3 2 0 2; do
  kubectl -n $NS scale statefulset/vgate-worker --replicas=$n
  claim "scale to $n: gateway sees $n healthy workers" wait_ready_workers $n
done
claim "chat after scaling back up" chat 3
echo "failures: $FAILS"
exit $FAILS
