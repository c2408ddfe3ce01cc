"""Build libwsmc.so (gfx950) in-tree with hipcc.

    python weightedsampling.jl_amd/build.py [--force] [--verbose]

Flags that matter for parity: -ffp-contract=off (no silent FMA contraction, so the
device evaluates the same IEEE operation sequence as the gcc-built oracle) and no
fast-math. The library lands next to the Python package (wsmc/libwsmc.so) so it ships
to the GPU box with the repo snapshot.
"""
from __future__ import annotations

import argparse
import os
import pathlib
import shutil
import subprocess
import sys
from concurrent.futures import ThreadPoolExecutor

PKG = pathlib.Path(__file__).resolve().parent
REPO = PKG.parent
CSRC = PKG / "csrc"
INCLUDE = REPO / "include"
OUT = PKG / "wsmc" / "libwsmc.so"
OBJDIR = PKG / "build"
SOURCES = ["wsmc_kernels.hip", "wsmc_api.hip", "wsmc_multi.hip"]
ARCH = os.environ.get("WSMC_OFFLOAD_ARCH", "gfx950")


def hipcc() -> str:
    for cand in (os.environ.get("HIPCC"), "/opt/rocm/bin/hipcc", shutil.which("hipcc")):
        if cand and pathlib.Path(cand).exists():
            return cand
    raise RuntimeError("hipcc not found")


COMMON = ["-O3", "-std=c++17", "-fPIC", "-ffp-contract=off", "-fno-fast-math",
          f"--offload-arch={ARCH}", "-I", str(INCLUDE), "-I", str(CSRC),
          "-Wno-unused-result", "-munsafe-fp-atomics"]


def _deps():
    return [CSRC / s for s in SOURCES] + list(CSRC.glob("*.h")) + list(INCLUDE.glob("*.h"))


def up_to_date() -> bool:
    if not OUT.exists():
        return False
    t = OUT.stat().st_mtime
    return all(p.stat().st_mtime <= t for p in _deps())


def build(force: bool = False, verbose: bool = False) -> pathlib.Path:
    if not force and up_to_date():
        return OUT
    OBJDIR.mkdir(exist_ok=True)
    cc = hipcc()

    def compile_one(src: str) -> pathlib.Path:
        obj = OBJDIR / (pathlib.Path(src).stem + ".o")
        cmd = [cc, *COMMON, "-c", str(CSRC / src), "-o", str(obj)]
        if verbose:
            print(" ".join(cmd), flush=True)
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError(f"hipcc failed on {src}:\n{r.stdout}\n{r.stderr}")
        if verbose and r.stderr:
            print(r.stderr, file=sys.stderr)
        return obj

    with ThreadPoolExecutor(max_workers=len(SOURCES)) as ex:
        objs = list(ex.map(compile_one, SOURCES))
    tmp = OUT.with_suffix(".so.tmp")
    cmd = [cc, f"--offload-arch={ARCH}", "-shared", "-fPIC", *map(str, objs), "-o", str(tmp),
           "-L/opt/rocm/lib", "-lrccl", "-Wl,-rpath,/opt/rocm/lib"]
    if verbose:
        print(" ".join(cmd), flush=True)
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"link failed:\n{r.stdout}\n{r.stderr}")
    os.replace(tmp, OUT)
    return OUT


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--force", action="store_true")
    ap.add_argument("--verbose", action="store_true")
    a = ap.parse_args()
    print(build(force=a.force, verbose=a.verbose))
