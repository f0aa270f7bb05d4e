"""Pull a model through zest (peers first, CDN fallback) and load it with transformers.

    python examples/download_model.py openai-community/gpt2
"""
import sys

import zest_amd as zest

repo = sys.argv[1] if len(sys.argv) > 1 else "openai-community/gpt2"
path = zest.pull(repo)
print("snapshot:", path)
try:
    from transformers import AutoModelForCausalLM, AutoTokenizer

    tok = AutoTokenizer.from_pretrained(path)
    model = AutoModelForCausalLM.from_pretrained(path)
    out = model.generate(**tok("The quick brown fox", return_tensors="pt"), max_new_tokens=20)
    print(tok.decode(out[0]))
except Exception as e:  # transformers optional
    print("transformers load skipped:", e)
