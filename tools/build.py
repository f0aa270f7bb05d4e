#!/usr/bin/env python3
"""Native build for zest_amd: host C++ core, HIP/CDNA4 kernels (gfx950), pybind11 modules, CLI.

Everything is built IN-TREE so the artefacts travel with the repo snapshot to the GPU box:

  zest_amd/_core.<abi>.so   host core (codecs, Xet, BT/DHT/HTTP stack, storage, swarm)  [g++]
  zest_amd/_hip.<abi>.so    HIP kernels + launchers for MI355X (gfx950)                 [hipcc]
  zest_amd/_bin/zest        native CLI (pull/seed/serve/start/stop/bench/version/help)  [g++]

Incremental: an object is rebuilt when its source or any header under csrc/ is newer.
Usage: python tools/build.py [--jobs N] [--clean] [--only core|hip|cli] [--debug] [--asan | --tsan]
"""
from __future__ import annotations

import argparse
import concurrent.futures as cf
import os
import shutil
import subprocess
import sys
import sysconfig
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
CSRC = ROOT / "csrc"
BUILD = ROOT / "build"
PKG = ROOT / "zest_amd"
ROCM = Path(os.environ.get("ROCM_PATH", "/opt/rocm"))
ARCH = os.environ.get("PYTORCH_ROCM_ARCH", "gfx950")
EXT = sysconfig.get_config_var("EXT_SUFFIX") or ".so"


def _pybind_include() -> str:
    import pybind11

    return pybind11.get_include()


def _py_include() -> str:
    return sysconfig.get_paths()["include"]


def _newest_header() -> float:
    t = 0.0
    for p in CSRC.rglob("*"):
        if p.suffix in (".h", ".hpp", ".cuh") and p.is_file():
            t = max(t, p.stat().st_mtime)
    return t


def _run(cmd: list[str]) -> None:
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        sys.stderr.write(" ".join(cmd) + "\n" + r.stdout + r.stderr)
        raise SystemExit(f"build failed: {cmd[-1] if cmd else ''}")


class Builder:
    def __init__(self, jobs: int, debug: bool, san: str = ""):
        self.jobs = jobs
        self.debug = debug
        self.hdr_time = _newest_header()
        opt = ["-O0", "-g"] if debug else ["-O1", "-g"] if san == "tsan" else ["-O3", "-g1"]
        san = {"asan": ["-fsanitize=address,undefined", "-fno-omit-frame-pointer"],
               "tsan": ["-fsanitize=thread", "-fno-omit-frame-pointer"]}.get(san, [])
        self.cxxflags = ["-std=c++17", "-fPIC", "-Wall", "-Wno-unused-function", "-pthread",
                         "-march=x86-64-v2", "-mtune=generic", f"-I{CSRC}", f"-I{CSRC / 'core'}",
                         f"-I{ROCM / 'include'}", "-D__HIP_PLATFORM_AMD__=1"] + opt + san
        self.ldflags = ["-pthread"] + san
        self.hipflags = ["-std=c++17", "-fPIC", f"--offload-arch={ARCH}", "-O3", "-g1",
                         "-Wno-unused-result", f"-I{CSRC}", f"-I{CSRC / 'core'}", f"-I{CSRC / 'gpu'}",
                         "-munsafe-fp-atomics"]

    def _stale(self, src: Path, obj: Path) -> bool:
        if not obj.exists():
            return True
        ot = obj.stat().st_mtime
        return src.stat().st_mtime > ot or self.hdr_time > ot

    def compile(self, srcs: list[Path], subdir: str, hip: bool = False, extra: list[str] | None = None) -> list[Path]:
        outdir = BUILD / subdir
        outdir.mkdir(parents=True, exist_ok=True)
        jobs = []
        objs = []
        for s in srcs:
            o = outdir / (s.stem + ".o")
            objs.append(o)
            if self._stale(s, o):
                if hip:
                    cmd = [str(ROCM / "bin" / "hipcc"), *self.hipflags, *(extra or []), "-c", str(s), "-o", str(o)]
                else:
                    cmd = ["g++", *self.cxxflags, *(extra or []), "-c", str(s), "-o", str(o)]
                jobs.append(cmd)
        if jobs:
            with cf.ThreadPoolExecutor(self.jobs) as ex:
                list(ex.map(_run, jobs))
        return objs

    def link(self, objs: list[Path], out: Path, shared: bool, libs: list[str], hip: bool = False) -> None:
        if out.exists() and all(o.stat().st_mtime <= out.stat().st_mtime for o in objs):
            return
        out.parent.mkdir(parents=True, exist_ok=True)
        tmp = out.with_name(out.name + ".tmp")
        if hip:
            cmd = [str(ROCM / "bin" / "hipcc"), f"--offload-arch={ARCH}", "-fPIC"]
        else:
            cmd = ["g++"]
        cmd += (["-shared"] if shared else []) + [str(o) for o in objs] + self.ldflags + libs + ["-o", str(tmp)]
        _run(cmd)
        os.replace(tmp, out)


def core_sources() -> list[Path]:
    return sorted((CSRC / "core").glob("*.cpp"))


def build(only: str | None = None, jobs: int | None = None, debug: bool = False, asan: bool = False,
          tsan: bool = False) -> dict:
    jobs = jobs or min(16, os.cpu_count() or 4)
    san = "asan" if asan else "tsan" if tsan else ""
    b = Builder(jobs, debug, san)
    built = {}
    if san:
        # Host-only sanitizer build (ASan + UBSan, or TSan) of the core, CLI and native unit tests,
        # kept out of the package: python tools/build.py --asan && build/asan/core_tests
        core_objs = b.compile(core_sources(), f"{san}/core")
        t_objs = b.compile(sorted((ROOT / "tests" / "cpp").glob("*.cpp")), f"{san}/tests")
        b.link(t_objs + core_objs, BUILD / san / "core_tests", shared=False, libs=["-lssl", "-lcrypto"])
        cli_objs = b.compile(sorted((CSRC / "cli").glob("*.cpp")), f"{san}/cli")
        b.link(cli_objs + core_objs, BUILD / san / "zest", shared=False, libs=["-lssl", "-lcrypto", "-ldl"])
        return {f"{san}_tests": BUILD / san / "core_tests", f"{san}_cli": BUILD / san / "zest"}
    core_objs = b.compile(core_sources(), "core")
    ssl_libs = ["-lssl", "-lcrypto"]
    if only in (None, "core"):
        bind_srcs = sorted(p for p in (CSRC / "bind").glob("*.cpp") if not p.name.startswith("hip_"))
        bind = b.compile(bind_srcs, "bind",
                         extra=[f"-I{_pybind_include()}", f"-I{_py_include()}", "-fvisibility=hidden"])
        out = PKG / f"_core{EXT}"
        b.link(core_objs + bind, out, shared=True, libs=ssl_libs)
        built["core"] = out
    if only in (None, "hip"):
        gpu_srcs = sorted((CSRC / "gpu").glob("*.hip"))
        gpu_objs = b.compile(gpu_srcs, "gpu", hip=True)
        hbind = b.compile(sorted((CSRC / "bind").glob("hip_*.cpp")), "hbind", hip=True,
                          extra=[f"-I{_pybind_include()}", f"-I{_py_include()}", "-fvisibility=hidden"])
        # native GPU runtime (device-direct pull): shared by the pybind module and the worker binary
        rt_srcs = sorted(p for p in (CSRC / "gpurt").glob("*.cpp") if p.name != "gpu_worker.cpp")
        rt_objs = b.compile(rt_srcs, "gpurt", hip=True)
        hip_libs = [f"-L{ROCM / 'lib'}", "-lamdhip64", f"-Wl,-rpath,{ROCM / 'lib'}"] + ssl_libs
        out = PKG / f"_hip{EXT}"
        b.link(gpu_objs + rt_objs + hbind + core_objs, out, shared=True, libs=hip_libs, hip=True)
        built["hip"] = out
        worker = CSRC / "gpurt" / "gpu_worker.cpp"
        if worker.exists():  # `zest pull --gpus N` worker: one process per GPU, no Python on its path
            w_objs = b.compile([worker], "gpurt", hip=True)
            out = PKG / "_bin" / "zest-gpu-worker"
            b.link(w_objs + rt_objs + gpu_objs + core_objs, out, shared=False, libs=hip_libs, hip=True)
            built["gpu_worker"] = out
    if only in (None, "cli"):
        cli_srcs = sorted((CSRC / "cli").glob("*.cpp"))
        if cli_srcs:
            cli_objs = b.compile(cli_srcs, "cli")
            out = PKG / "_bin" / "zest"
            b.link(cli_objs + core_objs, out, shared=False, libs=ssl_libs + ["-ldl"])
            built["cli"] = out
    if only in (None, "tests"):
        t_objs = b.compile(sorted((ROOT / "tests" / "cpp").glob("*.cpp")), "tests")
        if t_objs:
            out = BUILD / "tests" / "core_tests"
            b.link(t_objs + core_objs, out, shared=False, libs=ssl_libs)
            built["tests"] = out
    return built


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--jobs", type=int, default=None)
    ap.add_argument("--clean", action="store_true")
    ap.add_argument("--only", choices=["core", "hip", "cli", "tests"], default=None)
    ap.add_argument("--debug", action="store_true")
    ap.add_argument("--asan", action="store_true", help="host-only ASan/UBSan build of core + cli")
    ap.add_argument("--tsan", action="store_true", help="host-only ThreadSanitizer build of core + cli")
    a = ap.parse_args()
    if a.clean and BUILD.exists():
        shutil.rmtree(BUILD)
    out = build(a.only, a.jobs, a.debug, a.asan, a.tsan)
    for k, v in out.items():
        print(f"built {k}: {v.relative_to(ROOT)}")


if __name__ == "__main__":
    main()
