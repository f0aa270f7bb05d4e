"""Stand-in for the per-GPU worker of `zest pull --gpus N` in the elastic tests (no GPU needed).

The CLI starts one worker per device with ZEST_GPU_RANK / ZEST_GPU_WORLD / ZEST_GPU_STATUS and
HIP_VISIBLE_DEVICES pinned to that device (ZEST_GPU_DEVICES = the attempt's whole list).
ZEST_STUB_MODE=lose-last: in a multi-worker attempt the highest rank dies like a lost GPU, the
others finish; a single-worker attempt succeeds.  ZEST_STUB_MODE=always-crash: every worker dies,
so the CLI falls back to the host pull.  Worker 0 appends "<world>@<devices>" to ZEST_STUB_LOG.
"""
import json
import os


def main() -> int:
    rank = int(os.environ["ZEST_GPU_RANK"])
    world = int(os.environ["ZEST_GPU_WORLD"])
    if rank == 0:
        with open(os.environ["ZEST_STUB_LOG"], "a") as fh:
            fh.write(f"{world}@{os.environ['ZEST_GPU_DEVICES']}\n")
    with open(os.environ["ZEST_STUB_LOG"] + ".vis", "a") as fh:  # each worker sees one device
        fh.write(os.environ.get("HIP_VISIBLE_DEVICES", "") + "\n")
    mode = os.environ.get("ZEST_STUB_MODE", "lose-last")
    if mode == "always-crash" or (world > 1 and rank == world - 1):
        os._exit(17)
    with open(os.environ["ZEST_GPU_STATUS"], "w") as fh:
        json.dump({"complete": True, "rank": rank, "world": world, "failed_files": 0, "bytes": 0, "stats": {}}, fh)
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
