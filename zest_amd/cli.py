"""`zest` console entry point: run the bundled native binary.

Reference: python/zest/cli.py:1-43 replaces the interpreter with the binary (os.execv).  Here the
binary runs as a child process and its exit code is returned: replacing a process image is unsafe
once anything in it may have initialised the GPU (HIP runtime state does not survive exec).
"""
from __future__ import annotations

import signal
import subprocess
import sys

from .server import find_binary


def main(argv: list[str] | None = None) -> int:
    argv = sys.argv[1:] if argv is None else argv
    try:
        binary = find_binary()
    except FileNotFoundError as e:
        print(f"zest: {e}", file=sys.stderr)
        return 127
    proc = subprocess.Popen([binary, *argv])
    try:
        return proc.wait()
    except KeyboardInterrupt:
        proc.send_signal(signal.SIGINT)
        return proc.wait()


if __name__ == "__main__":
    sys.exit(main())
