"""NUMA binding helper (zest_amd.parallel.bind_local_numa) on CPU: cpulist parsing and the
intersection / no-op rules. The sysfs lookup itself runs on the GPU box in bench.py."""
import os

import pytest

from zest_amd.parallel import bind_local_numa, parse_cpulist


def test_parse_cpulist():
    assert parse_cpulist("0-3,8,10-11\n") == {0, 1, 2, 3, 8, 10, 11}
    assert parse_cpulist("") == set()
    assert parse_cpulist("5") == {5}


@pytest.mark.skipif(not hasattr(os, "sched_setaffinity"), reason="Linux only")
def test_bind_local_numa_intersects_and_restores():
    before = os.sched_getaffinity(0)
    try:
        # no overlap with the allowed set -> unchanged
        assert bind_local_numa(None, local_cpus={10 ** 6}) == []
        assert os.sched_getaffinity(0) == before
        # opt-out
        os.environ["ZEST_NUMA_BIND"] = "0"
        assert bind_local_numa(None, local_cpus=set(before)) == []
        del os.environ["ZEST_NUMA_BIND"]
        if len(before) > 1:
            one = {min(before)}
            assert bind_local_numa(None, local_cpus=one | {10 ** 6}) == sorted(one)
            assert os.sched_getaffinity(0) == one
    finally:
        os.environ.pop("ZEST_NUMA_BIND", None)
        os.sched_setaffinity(0, before)
