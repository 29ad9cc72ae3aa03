"""Build the host runtime library (``libdpc_runtime.so``) in-tree with g++ (OpenMP)."""
from __future__ import annotations

import os
import shutil
import subprocess
import sys
from pathlib import Path

HERE = Path(__file__).resolve().parent
SRC = HERE / "csrc" / "runtime.cpp"
LIB_PATH = HERE / "libdpc_runtime.so"
FLAGS = ["-O3", "-std=c++17", "-fPIC", "-shared", "-fopenmp", "-march=x86-64-v3", "-pthread"]


def needs_build() -> bool:
    return not LIB_PATH.exists() or SRC.stat().st_mtime > LIB_PATH.stat().st_mtime


def build(force: bool = False, verbose: bool = False) -> Path:
    if not force and not needs_build():
        return LIB_PATH
    cxx = os.environ.get("CXX") or shutil.which("g++") or shutil.which("c++")
    if not cxx:
        raise RuntimeError("no C++ compiler found for the host runtime")
    tmp = LIB_PATH.with_suffix(".so.tmp")
    cmd = [cxx, *FLAGS, str(SRC), "-o", str(tmp)]
    if verbose:
        print(" ".join(cmd), flush=True)
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"runtime build failed:\n{r.stdout}\n{r.stderr}")
    os.replace(tmp, LIB_PATH)
    return LIB_PATH


if __name__ == "__main__":
    print(build(force="--force" in sys.argv, verbose=True))
