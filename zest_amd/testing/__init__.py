"""Test fixtures: offline Hub/CAS/tracker fakes."""
from .fakehub import FakeHub

__all__ = ["FakeHub"]
