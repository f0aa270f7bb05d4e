#!/usr/bin/env bash
# Pull a model with zest (CDN only) into a fresh HF cache and run it with transformers: the
# reference's test/local/verify-model.sh.  Needs network + HF_TOKEN.  Offline equivalent (fake Hub,
# random-init GPT-2, exact logits check): tests/test_verify_model.py.
#
#   scripts/verify_model.sh [repo] [prompt]
set -euo pipefail
REPO="${1:-openai-community/gpt2}"
PROMPT="${2:-The quick brown fox}"
ROOT="$(cd "$(dirname "$0")/.." && pwd)"
ZEST="${ZEST_BIN:-$ROOT/zest_amd/_bin/zest}"
[[ -x "$ZEST" ]] || python3 "$ROOT/tools/build.py" --only cli
python3 -c "import transformers, torch" || { echo "[FAIL] needs transformers + torch"; exit 1; }
TMP="$(mktemp -d /tmp/zest-verify-XXXXXX)"
trap 'rm -rf "$TMP"' EXIT
export HF_HOME="$TMP/hf" HF_HUB_CACHE="$TMP/hf/hub" ZEST_CACHE_DIR="$TMP/zest" ZEST_NO_AUTOSTART=1
"$ZEST" pull "$REPO" --no-p2p | tee "$TMP/pull.log"
SNAP="$(dirname "$(find "$HF_HUB_CACHE" -name config.json | head -1)")"
[[ -d "$SNAP" ]] || { echo "[FAIL] no snapshot"; exit 1; }
HF_HUB_OFFLINE=1 TRANSFORMERS_OFFLINE=1 python3 - "$SNAP" "$PROMPT" <<'PY'
import sys, torch
from transformers import AutoModelForCausalLM, AutoTokenizer
path, prompt = sys.argv[1], sys.argv[2]
tok = AutoTokenizer.from_pretrained(path)
model = AutoModelForCausalLM.from_pretrained(path, torch_dtype=torch.float32).eval()
n = sum(p.numel() for p in model.parameters())
out = model.generate(**tok(prompt, return_tensors="pt"), max_new_tokens=20, do_sample=False)
print(f"parameters: {n:,}")
print("output:", tok.decode(out[0], skip_special_tokens=True))
assert n > 1_000_000
PY
echo "[PASS] $REPO pulled by zest loads and generates"
