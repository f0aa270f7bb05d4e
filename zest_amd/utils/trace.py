"""Python spans in the same trace as the C++ core (csrc/core/trace.h).

ZEST_TRACE=1 prints span lines on stderr; ZEST_TRACE=/path/trace.json writes a Chrome trace-event
file at exit containing host spans from C++ (pull, CDN fetches, peer requests) and Python, plus
device spans measured with HIP events (`device_span`) placed on the host timeline.
ZEST_ROCTX=1 additionally turns every span (C++ and Python) into a roctx range, so
`rocprofv3 --marker-trace` shows the pull phases alongside the kernels.
"""
from __future__ import annotations

import contextlib
import json

from .. import _core

_tr = _core.trace


def trace_enabled() -> bool:
    return _tr.enabled()


class Span:
    """Host span: `with Span("engine", "round 3", bytes=123): ...`"""

    def __init__(self, cat: str, name: str, **args):
        self.cat, self.name, self.args = cat, name, args
        self.on = _tr.enabled()
        self.rx = _tr.roctx_enabled()

    def __enter__(self):
        if self.rx:
            _tr.roctx_push(f"{self.cat}: {self.name}")
        if self.on:
            self.t0 = _tr.now_us()
        return self

    def __exit__(self, *exc):
        if self.rx:
            _tr.roctx_pop()
        if self.on:
            _tr.complete(self.cat, self.name, self.t0, _tr.now_us() - self.t0,
                         json.dumps(self.args)[1:-1] if self.args else "")
        return False


@contextlib.contextmanager
def device_span(cat: str, name: str, stream=None, **args):
    """Times the enclosed GPU work with HIP events; records it as a span on the host timeline
    (synchronizes the stream at exit, so use it for coarse phases only)."""
    if not _tr.enabled():
        yield
        return
    import torch

    s = stream or torch.cuda.current_stream()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    t0 = _tr.now_us()
    e0.record(s)
    try:
        yield
    finally:
        e1.record(s)
        e1.synchronize()
        dur = int(e0.elapsed_time(e1) * 1000)
        _tr.complete(cat, name + " [gpu]", t0, dur, json.dumps(args)[1:-1] if args else "")
