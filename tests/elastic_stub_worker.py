"""Stand-in for zest_amd.multigpu in the elastic `zest pull --gpus N` tests (no GPU needed).

ZEST_STUB_MODE=lose-last: in a multi-rank attempt the highest rank dies like a lost GPU (rank 0
waits, so torchrun stops it before it can report completion); a single-rank attempt succeeds.
ZEST_STUB_MODE=always-crash: every attempt dies, so the CLI falls back to the host pull.
Each attempt appends its world size (and HIP_VISIBLE_DEVICES, when the CLI set one) to ZEST_STUB_LOG.
"""
import json
import os
import time


def main() -> int:
    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    # all ranks of one attempt are children of the same torchrun agent
    ready = f"{os.environ['ZEST_STUB_LOG']}.ready.{os.getppid()}"
    if rank == 0:
        with open(os.environ["ZEST_STUB_LOG"], "a") as fh:
            vis = os.environ.get("HIP_VISIBLE_DEVICES")
            fh.write(f"{world}" + (f"@{vis}" if vis else "") + "\n")
        open(ready, "w").close()
    mode = os.environ.get("ZEST_STUB_MODE", "lose-last")
    if mode == "always-crash" or (world > 1 and rank == world - 1):
        # die only after rank 0 logged the attempt (torchrun stops rank 0 as soon as a peer dies)
        t0 = time.time()
        while rank != 0 and not os.path.exists(ready) and time.time() - t0 < 60:
            time.sleep(0.01)
        os._exit(17)
    if world > 1:
        time.sleep(60)  # never reached in the tests: torchrun tears the group down first
    if rank == 0:
        with open(os.environ["ZEST_GPU_STATUS"], "w") as fh:
            json.dump({"complete": True, "world": world, "failed_files": 0}, fh)
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
