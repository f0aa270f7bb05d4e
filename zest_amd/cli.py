"""`zest` console entry point: run the bundled native binary.

`zest pull <repo> --gpus N --device all` is handled in Python (zest_amd.replicate): N rank processes,
each ending with the whole model verified in its GPU's memory.

Reference: python/zest/cli.py:1-43 replaces the interpreter with the binary (os.execv).  Here the
binary runs as a child process and its exit code is returned: replacing a process image is unsafe
once anything in it may have initialised the GPU (HIP runtime state does not survive exec).
"""
from __future__ import annotations

import signal
import subprocess
import sys

from .server import find_binary


def _device_all(argv: list[str]) -> bool:
    return any(x == "--device=all" or (x == "--device" and i + 1 < len(argv) and argv[i + 1] == "all")
               for i, x in enumerate(argv))


def main(argv: list[str] | None = None) -> int:
    argv = sys.argv[1:] if argv is None else argv
    if argv[:1] == ["pull"] and _device_all(argv):
        # `zest pull <repo> --gpus N --device all`: every tensor resident on every GPU, one rank per
        # GPU (zest_amd.replicate; the launcher starts the ranks before anything touches a GPU)
        from .replicate import main as replicate_main
        return replicate_main(argv[1:])
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
