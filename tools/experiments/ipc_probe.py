"""Time HIP IPC export/import of large HBM allocations between two processes on one GPU
(torch reduce_tensor / rebuild), to size the `ipc`/`xgmi` exchange's setup cost."""
import os
import sys
import time

import torch
import torch.multiprocessing as mp


def child(q_in, q_out):
    torch.cuda.set_device(0)
    while True:
        item = q_in.get()
        if item is None:
            return
        gb, (fn, args) = item
        t = time.time()
        x = fn(*args)
        torch.cuda.synchronize()
        v = int(x[-1].item())
        q_out.put((gb, time.time() - t, v))
        del x


def main():
    sizes = [float(s) for s in (sys.argv[1:] or ["0.25", "1", "4", "16"])]
    ctx = mp.get_context("spawn")
    qi, qo = ctx.Queue(), ctx.Queue()
    p = ctx.Process(target=child, args=(qi, qo))
    p.start()
    torch.cuda.set_device(0)
    from torch.multiprocessing.reductions import reduce_tensor
    for gb in sizes:
        t = torch.empty(int(gb * (1 << 30)), dtype=torch.uint8, device="cuda:0")
        t[-1] = 7
        torch.cuda.synchronize()
        t0 = time.time()
        h = reduce_tensor(t)
        t_exp = time.time() - t0
        qi.put((gb, h))
        r = qo.get(timeout=300)
        print(f"{gb:6.2f} GiB: export {t_exp:.3f}s import+touch {r[1]:.3f}s value {r[2]}", flush=True)
        del t
        torch.cuda.empty_cache()
    qi.put(None)
    p.join(timeout=60)


if __name__ == "__main__":
    main()
