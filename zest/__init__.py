"""Compatibility package: `import zest` exposes the zest_amd API (enable/disable/pull/status/stop,
plus from_pretrained), so code written against the reference's Python package runs unchanged."""
from zest_amd import __version__, disable, enable, from_pretrained, pull, status, stop  # noqa: F401

__all__ = ["__version__", "disable", "enable", "from_pretrained", "pull", "status", "stop"]
