"""Build the host runtime library (``libdpc_runtime.so``) in-tree with g++ (OpenMP).

Sources: ``csrc/runtime.cpp`` (token-file loader, synthetic corpus, host AdamW) and
``csrc/rccl_comm.cpp`` (native RCCL communicator, resolved at run time with dlopen).
"""
from __future__ import annotations

import os
import shutil
import subprocess
import sys
from pathlib import Path

HERE = Path(__file__).resolve().parent
SRCS = [HERE / "csrc" / "runtime.cpp", HERE / "csrc" / "rccl_comm.cpp"]
LIB_PATH = HERE / "libdpc_runtime.so"
FLAGS = ["-O3", "-std=c++17", "-fPIC", "-shared", "-fopenmp", "-march=x86-64-v3", "-pthread"]
LIBS = ["-ldl"]


HASH_PATH = LIB_PATH.with_suffix(".so.srchash")


def source_hash() -> str:
    import hashlib

    h = hashlib.sha256(" ".join(FLAGS + LIBS).encode())
    for src in SRCS:
        h.update(src.name.encode())
        h.update(src.read_bytes())
    return h.hexdigest()


def needs_build() -> bool:
    if not LIB_PATH.exists() or not HASH_PATH.exists():
        return True
    return HASH_PATH.read_text().strip() != source_hash()


def build(force: bool = False, verbose: bool = False) -> Path:
    if not force and not needs_build():
        return LIB_PATH
    cxx = os.environ.get("CXX") or shutil.which("g++") or shutil.which("c++")
    if not cxx:
        raise RuntimeError("no C++ compiler found for the host runtime")
    tmp = LIB_PATH.with_suffix(".so.tmp")
    cmd = [cxx, *FLAGS, *map(str, SRCS), "-o", str(tmp), *LIBS]
    if verbose:
        print(" ".join(cmd), flush=True)
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"runtime build failed:\n{r.stdout}\n{r.stderr}")
    os.replace(tmp, LIB_PATH)
    HASH_PATH.write_text(source_hash() + "\n")
    return LIB_PATH


if __name__ == "__main__":
    print(build(force="--force" in sys.argv, verbose=True))
