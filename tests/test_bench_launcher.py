"""bench.py contract on CPU: `python bench.py --gpus N` launches its own ranks (torchrun child),
prints one JSON line, and a rank that hangs ends the run with a non-zero status instead of a
silent empty record (per-phase watchdog, launcher timeout)."""
import json
import os
import subprocess
import sys
import time

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BENCH = os.path.join(ROOT, "bench.py")


def _run(args, env_extra=None, timeout=240):
    env = dict(os.environ)
    env.pop("WORLD_SIZE", None)
    env.pop("RANK", None)
    env.update(env_extra or {})
    t0 = time.time()
    p = subprocess.run([sys.executable, BENCH, "--device", "cpu", "--model", "llama-tiny", *args],
                       capture_output=True, text=True, timeout=timeout, env=env, cwd=ROOT)
    return p, time.time() - t0


def _json_lines(text):
    return [json.loads(ln) for ln in text.splitlines() if ln.startswith("{")]


@pytest.mark.parametrize("gpus", [1, 2])
def test_bench_prints_one_json_line(gpus):
    p, _ = _run(["--gpus", str(gpus), "--steps", "2", "--warmup", "1"])
    assert p.returncode == 0, p.stderr[-3000:]
    lines = _json_lines(p.stdout)
    assert len(lines) == 1, p.stdout
    out = lines[0]
    assert out["n_gpus"] == gpus and out["steps"] == 2 and out["warmup"] == 1
    assert out["metric"].startswith("aggregate pull GB/s")
    assert out["value"] > 0 and out["higher_is_better"] is True
    # both data modes measured; the first (bf16) is the headline
    assert out["config"]["modes"] == ["bf16", "random"]
    assert out["extra"]["bf16_GBps"] == out["value"] and out["extra"]["random_GBps"] > 0
    # self-validation: ranks the collective counted, the devices behind them, per-phase seconds
    cfg = out["config"]
    assert cfg["rccl_ranks"] == gpus and cfg["devices"] == ["cpu"] * gpus and cfg["distinct_devices"] is False
    assert set(cfg["phase_s"]) >= {"world_s", "origin_s", "setup_s", "autotune_s", "warmup_s", "timed_s"}
    assert len(cfg["exchange_rx_GBps"]) == gpus
    if gpus > 1:
        assert out["config"]["backend"] == "gloo" and 0 < out["p2p_ratio"] < 1
        assert "launching 2 ranks" in p.stderr
        assert sum(cfg["exchange_rx_GBps"]) > 0


def test_bench_one_seeder_one_leecher():
    """BASELINE config 2's shape: rank 0 pulls everything from the origin, rank 1 leeches it all
    from rank 0 (half of the job's bytes arrive from a peer)."""
    p, _ = _run(["--gpus", "2", "--seeders", "1", "--steps", "2", "--warmup", "1", "--modes", "random"])
    assert p.returncode == 0, p.stderr[-3000:]
    out = _json_lines(p.stdout)[0]
    assert out["config"]["parallelism"] == "seed1-leech1"
    assert abs(out["p2p_ratio"] - 0.5) < 1e-6 and out["value"] > 0


def test_bench_hung_rank_fails_fast():
    """Rank 1 stops in the warm-up phase: its watchdog dumps the stack and exits, torchrun tears
    rank 0 down, and the launcher returns non-zero well before any driver timeout."""
    p, dt = _run(["--gpus", "2", "--steps", "1", "--warmup", "1", "--modes", "random"],
                 {"ZEST_BENCH_WATCHDOG": "8", "ZEST_BENCH_FAULT": "hang:1:warmup", "ZEST_BENCH_PG_TIMEOUT": "20"})
    assert p.returncode != 0
    assert not _json_lines(p.stdout)
    assert "Timeout" in p.stderr or "most recent call first" in p.stderr, p.stderr[-3000:]
    assert dt < 150


def test_bench_launcher_timeout_kills_group():
    """Watchdog disabled: the launcher's own deadline kills the whole rank group (exit 124)."""
    p, dt = _run(["--gpus", "2", "--steps", "1", "--warmup", "1", "--modes", "random"],
                 {"ZEST_BENCH_WATCHDOG": "0", "ZEST_BENCH_FAULT": "hang:1:timed", "ZEST_BENCH_TIMEOUT": "25"})
    assert p.returncode == 124, p.stderr[-2000:]
    assert dt < 90


@pytest.mark.parametrize("gpus", [1, 2])
def test_bench_swarm_row_times_the_public_path(gpus):
    """--swarm-row on: after each engine mode, the same world is pulled through the public
    swarm_pull path from a mem:// memory CAS (every rank's pinned origin); extra.swarm_pull_* reports
    the first mode's row and swarm_pull_<mode>_* every mode's -- here on gloo CPU ranks."""
    p, _ = _run(["--gpus", str(gpus), "--steps", "2", "--warmup", "1", "--modes", "random,bf16", "--swarm-row", "on",
                 "--swarm-steps", "2", "--swarm-warmup", "1"])
    assert p.returncode == 0, p.stderr[-3000:]
    lines = _json_lines(p.stdout)
    assert len(lines) == 1, p.stdout
    ex = lines[0]["extra"]
    assert ex["swarm_pull_GBps"] > 0 and len(ex["swarm_pull_step_s"]) == 2
    assert ex["swarm_pull_arena_reused"]  # timed pulls land in the warm-up pull's arena
    assert ex["swarm_pull_mode"] == "random" and ex["swarm_pull_tensors"] > 0
    assert ex["swarm_pull_fetch"]["bytes_from_cdn"] > 0 and not ex["swarm_pull_fetch"]["bytes_from_peer"]
    if gpus > 1:
        assert ex["swarm_pull_p2p_ratio"] > 0.3 and ex["swarm_pull_exchange"] in ("bcast", "allgather", "p2p")
    for mode in ("random", "bf16"):  # the row ran on both worlds, each against its own engine number
        assert ex[f"swarm_pull_{mode}_GBps"] > 0
        assert ex[f"swarm_pull_{mode}_vs_engine"] == pytest.approx(ex[f"swarm_pull_{mode}_GBps"] / ex[f"{mode}_GBps"], rel=1e-2)
        assert len(ex["swarm_pull_modes"][mode]["step_s"]) == 2


def test_bench_swarm_row_multi_file_three_ranks():
    """Three ranks on a 10-file model: the swarm row's term split matches the engine's per-rank
    origin shares (every rank's CDN fetches are served by its own memory CAS)."""
    p, _ = _run(["--gpus", "3", "--steps", "1", "--warmup", "1", "--modes", "random", "--swarm-row", "on",
                 "--swarm-steps", "1", "--swarm-warmup", "1", "--model", "llama-tiny-sharded"])
    assert p.returncode == 0, p.stderr[-3000:]
    lines = _json_lines(p.stdout)
    assert len(lines) == 1, p.stdout
    ex = lines[0]["extra"]
    assert "swarm_pull_error" not in ex and ex["swarm_pull_GBps"] > 0
    assert ex["swarm_pull_p2p_ratio"] > 0.5  # each rank received the other two thirds
    assert ex["swarm_pull_arena_reused"]


def test_bench_swarm_row_overrun_keeps_the_headline():
    """A rank that hangs inside the swarm row (after the headline was measured): the row's deadline
    prints the headline line once, with extra.swarm_pull_error, and every rank exits 0."""
    p, dt = _run(["--gpus", "2", "--steps", "1", "--warmup", "1", "--modes", "random", "--swarm-row", "on",
                  "--swarm-steps", "1", "--swarm-warmup", "1"],
                 env_extra={"ZEST_BENCH_FAULT": "hang:1:swarm_timed", "ZEST_BENCH_WATCHDOG": "25"})
    assert p.returncode == 0, p.stderr[-3000:]
    lines = _json_lines(p.stdout)
    assert len(lines) == 1, p.stdout
    assert lines[0]["value"] > 0 and "swarm_timed" in lines[0]["extra"]["swarm_pull_error"]
    assert "swarm_pull_GBps" not in lines[0]["extra"]


def test_swarm_extra_reports_each_mode_and_errors():
    """_swarm_extra: the first mode's row under swarm_pull_*, every mode's throughput and its ratio to
    the engine on the same world under swarm_pull_<mode>_*, a failed mode's error under
    swarm_pull_<mode>_error (and no throughput for it)."""
    import importlib.util
    import os
    spec = importlib.util.spec_from_file_location("bench_mod", os.path.join(os.path.dirname(os.path.dirname(
        os.path.abspath(__file__))), "bench.py"))
    bench = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(bench)
    rows = {"bf16": {"swarm_pull_GBps": 62.0, "swarm_pull_ms_per_step": 2270.0, "swarm_pull_step_s": [2.27],
                     "swarm_pull_streamed": False, "swarm_pull_exchange": "none"},
            "random": {"swarm_pull_error": "RuntimeError: boom"}}
    results = [{"mode": "bf16", "value": 64.0}, {"mode": "random", "value": 56.0}]
    ex = bench._swarm_extra(rows, results)
    assert ex["swarm_pull_GBps"] == 62.0 and ex["swarm_pull_bf16_GBps"] == 62.0
    assert ex["swarm_pull_bf16_vs_engine"] == round(62.0 / 64.0, 4)
    assert ex["swarm_pull_random_error"] == "RuntimeError: boom"
    assert "swarm_pull_random_GBps" not in ex and set(ex["swarm_pull_modes"]) == {"bf16"}
    assert bench._swarm_extra({}, results) == {}
