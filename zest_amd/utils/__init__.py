"""Utilities: tracing spans shared with the native core, fault-injection specs, formatting."""
from .fault import FaultSpec
from .fmt import human_bytes, human_rate
from .trace import Span, device_span, trace_enabled

__all__ = ["FaultSpec", "Span", "device_span", "human_bytes", "human_rate", "trace_enabled"]
