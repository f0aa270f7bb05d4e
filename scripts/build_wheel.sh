#!/bin/bash
# Build a wheel containing _core/_hip (gfx950) and the zest CLI.
set -euo pipefail
cd "$(dirname "$0")/.."
python tools/build.py
python -m pip wheel --no-deps --no-build-isolation -w dist .
ls -la dist
