#!/usr/bin/env bash
# P2P integration suite: a CDN-only baseline, then pulls from one and from all seeders, with a
# results table.  Same scenario as the reference's test/hetzner/p2p-test.sh and
# test/local/p2p-docker-test.sh, but it does not provision VMs or containers.  It runs on nodes
# you already have:
#
#   scripts/p2p_cluster_test.sh --local 3                       # 3 nodes on this host, offline fake Hub
#   scripts/p2p_cluster_test.sh --local 3 --repo openai-community/gpt2 --real-hub   # real Hub (HF_TOKEN)
#   scripts/p2p_cluster_test.sh --hosts gpu0,gpu1,gpu2 --repo meta-llama/Llama-3.1-8B  # over ssh
#
# Node 0 is the leecher.  Nodes 1..N-1 pull CDN-only and then `zest serve`.  Servers are stopped
# through their REST API (POST /v1/stop), never by process name.
set -euo pipefail

MODE=""; NLOCAL=3; HOSTS=""; REPO=""; REAL_HUB=0; BT_PORT=6881; HTTP_PORT=9847
ROOT="$(cd "$(dirname "$0")/.." && pwd)"
ZEST="${ZEST_BIN:-$ROOT/zest_amd/_bin/zest}"
while [[ $# -gt 0 ]]; do
  case "$1" in
    --local) MODE=local; NLOCAL="$2"; shift 2 ;;
    --hosts) MODE=ssh; HOSTS="$2"; shift 2 ;;
    --repo) REPO="$2"; shift 2 ;;
    --real-hub) REAL_HUB=1; shift ;;
    --bt-port) BT_PORT="$2"; shift 2 ;;
    --http-port) HTTP_PORT="$2"; shift 2 ;;
    -h|--help) sed -n 2,14p "$0"; exit 0 ;;
    *) echo "unknown argument: $1" >&2; exit 2 ;;
  esac
done
[[ -n "$MODE" ]] || { sed -n 2,14p "$0"; exit 2; }

info() { echo "[INFO] $*"; }
pass() { echo "[PASS] $*"; }
fail() { echo "[FAIL] $*"; exit 1; }

WORK="$(mktemp -d /tmp/zest-p2p-XXXXXX)"
HUB_PID=""; SERVERS=()
cleanup() {
  for s in "${SERVERS[@]:-}"; do [[ -n "$s" ]] && node_api "$s" /v1/stop POST >/dev/null 2>&1 || true; done
  [[ -n "$HUB_PID" ]] && kill "$HUB_PID" 2>/dev/null || true
  rm -rf "$WORK"
}
trap cleanup EXIT

# ---------------------------------------------------------------- node abstraction
if [[ "$MODE" == local ]]; then
  N="$NLOCAL"
  if [[ "$REAL_HUB" == 0 ]]; then
    info "starting the offline fake Hub"
    python3 -m zest_amd.testing ${REPO:+--repo "$REPO"} > "$WORK/hub.json" 2> "$WORK/hub.log" &
    HUB_PID=$!
    for _ in $(seq 100); do [[ -s "$WORK/hub.json" ]] && break; sleep 0.2; done
    [[ -s "$WORK/hub.json" ]] || fail "fake hub did not start: $(cat "$WORK/hub.log")"
    HUB_URL=$(python3 -c 'import json,sys; print(json.load(open(sys.argv[1]))["url"])' "$WORK/hub.json")
    REPO=$(python3 -c 'import json,sys; print(json.load(open(sys.argv[1]))["repo"])' "$WORK/hub.json")
    HUB_ENV="HF_ENDPOINT=$HUB_URL HF_TOKEN=hf_fake_token"
  else
    [[ -n "$REPO" ]] || fail "--real-hub needs --repo"
    HUB_ENV=""
  fi
  node_addr() { echo "127.0.0.1"; }
  node_bt() { echo $((BT_PORT + 10 * $1)); }
  node_http() { echo $((HTTP_PORT + 10 * $1)); }
  node_sh() {  # node_sh K command...
    local k="$1"; shift
    local h="$WORK/node$k"; mkdir -p "$h"
    env $HUB_ENV HOME="$h" HF_HOME="$h/hf" HF_HUB_CACHE="$h/hf/hub" ZEST_CACHE_DIR="$h/zest" ZEST_NO_AUTOSTART=1 \
      ZEST_LISTEN_PORT="$(node_bt "$k")" ZEST_HTTP_PORT="$(node_http "$k")" ZEST_DHT_PORT="$(( $(node_bt "$k") + 1 ))" \
      bash -c "$*"
  }
else
  IFS=, read -r -a HOSTLIST <<< "$HOSTS"
  N=${#HOSTLIST[@]}
  [[ -n "$REPO" ]] || fail "--hosts needs --repo"
  node_addr() { echo "${HOSTLIST[$1]#*@}"; }
  node_bt() { echo "$BT_PORT"; }
  node_http() { echo "$HTTP_PORT"; }
  node_sh() { local k="$1"; shift; ssh -o BatchMode=yes "${HOSTLIST[$k]}" "$*"; }
  ZEST="${ZEST_BIN:-zest}"
fi
(( N >= 2 )) || fail "need at least 2 nodes"
node_api() {  # node_api K path [method]
  node_sh "$1" "curl -s -X ${3:-GET} http://127.0.0.1:$(node_http "$1")$2"
}
clean_cache() { node_sh "$1" 'rm -rf "$HOME/.cache/zest" "$ZEST_CACHE_DIR" "$HF_HOME/hub" 2>/dev/null; true'; }
timed_pull() {  # timed_pull K logfile args...  -> prints seconds
  local k="$1" log="$2"; shift 2
  local t0 t1
  t0=$(date +%s.%N)
  node_sh "$k" "$ZEST pull $REPO $*" > "$log" 2>&1 || { cat "$log" >&2; fail "pull on node $k failed"; }
  t1=$(date +%s.%N)
  python3 -c "print(f'{$t1 - $t0:.2f}')"
}
ratio() { { grep -Eo 'P2P ratio: *[0-9.]+' "$1" || echo 0; } | grep -Eo '[0-9.]+$' | tail -1; }
snapshot_digest() {
  node_sh "$1" "cd \"\$HF_HOME/hub\"/models--*/snapshots/* && find . -type f -print0 | sort -z | xargs -0 sha256sum | sha256sum | cut -c1-16"
}

# ---------------------------------------------------------------- suite
info "repo: $REPO, nodes: $N ($MODE), zest: $ZEST"
clean_cache 0
T_CDN=$(timed_pull 0 "$WORK/cdn.log" --no-p2p)
pass "CDN-only baseline on node 0: ${T_CDN}s"
REF_DIGEST=$(snapshot_digest 0)

PEERS=()
for k in $(seq 1 $((N - 1))); do
  clean_cache "$k"
  timed_pull "$k" "$WORK/seed$k.log" --no-p2p > /dev/null
  node_sh "$k" "nohup $ZEST serve --listen-port $(node_bt "$k") --http-port $(node_http "$k") > \"\$HOME/zest-serve.log\" 2>&1 &"
  SERVERS+=("$k")
  for _ in $(seq 50); do node_api "$k" /v1/health 2>/dev/null | grep -q ok && break; sleep 0.2; done
  node_api "$k" /v1/health | grep -q ok || fail "seeder $k did not come up"
  PEERS+=(--peer "$(node_addr "$k"):$(node_bt "$k")")
  pass "node $k seeding on $(node_addr "$k"):$(node_bt "$k")"
done

clean_cache 0
T_ALL=$(timed_pull 0 "$WORK/p2p_all.log" "${PEERS[@]}" --no-dht)
R_ALL=$(ratio "$WORK/p2p_all.log")
[[ "$(snapshot_digest 0)" == "$REF_DIGEST" ]] || fail "snapshot differs after P2P pull (all peers)"
pass "P2P from $((N - 1)) peer(s): ${T_ALL}s, P2P ratio ${R_ALL}%"

clean_cache 0
T_ONE=$(timed_pull 0 "$WORK/p2p_one.log" --peer "$(node_addr 1):$(node_bt 1)" --no-dht)
R_ONE=$(ratio "$WORK/p2p_one.log")
[[ "$(snapshot_digest 0)" == "$REF_DIGEST" ]] || fail "snapshot differs after P2P pull (one peer)"
pass "P2P from 1 peer: ${T_ONE}s, P2P ratio ${R_ONE}%"

echo
echo "  +--------------------------------------------------+"
echo "  | zest P2P integration results                     |"
echo "  +--------------------------------------------------+"
printf "  | %-22s | %9s | %11s |\n" "scenario" "time (s)" "P2P ratio"
printf "  | %-22s | %9s | %11s |\n" "CDN only" "$T_CDN" "0%"
printf "  | %-22s | %9s | %10s%% |\n" "P2P, $((N - 1)) peer(s)" "$T_ALL" "$R_ALL"
printf "  | %-22s | %9s | %10s%% |\n" "P2P, 1 peer" "$T_ONE" "$R_ONE"
echo "  +--------------------------------------------------+"
python3 -c "import sys; sys.exit(0 if float('$R_ALL') > 0 and float('$R_ONE') > 0 else 1)" \
  || fail "no bytes came from peers"
pass "all scenarios passed"
