"""HBM bytes written per kernel launch from one rocprofv3 --pmc WRITE_SIZE pass (KiB in rocprof's
definition), e.g. k_lz4_pair with the BG4 staging on and off:

    python tools/gpu/pmc_write.py DIR [--kernel k_lz4_pair] [--output-bytes N]
"""
import argparse
import sys

sys.path.insert(0, __file__.rsplit("/", 1)[0])
from pmc_table import load, short  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dir")
    ap.add_argument("--kernel", default="k_lz4_pair")
    ap.add_argument("--output-bytes", type=float, default=0.0, help="bytes the kernel produces per launch")
    a = ap.parse_args()
    cnt, disp, dur = load(a.dir)
    for k, c in cnt.items():
        if a.kernel not in k or "WRITE_SIZE" not in c:
            continue
        n = max(1, len(disp[k]))
        wr = c["WRITE_SIZE"] / n * 1024
        us = sum(dur.get(k, [0])) / max(1, len(dur.get(k, [])))
        ratio = f", {wr / a.output_bytes:.2f}x the output" if a.output_bytes else ""
        print(f"{short(k)}: {n} launches, {us:.1f} us/launch, HBM written {wr / 1e6:.1f} MB/launch{ratio}")


if __name__ == "__main__":
    main()
