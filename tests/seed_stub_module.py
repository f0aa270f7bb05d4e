"""Stand-in for `python -m zest_amd.seed` in the CLI test of `zest seed --hbm-cache-gb` (no GPU):
records its argv in ZEST_STUB_LOG and exits 0."""
import json
import os
import sys

if __name__ == "__main__":
    with open(os.environ["ZEST_STUB_LOG"], "w") as fh:
        json.dump(sys.argv[1:], fh)
    raise SystemExit(0)
