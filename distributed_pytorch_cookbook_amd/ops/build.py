"""Build the gfx950 kernel library (``libdpc_kernels.so``) in-tree with hipcc.

The kernels are plain HIP C++ with a C ABI (no torch headers, no hipify, no
``torch.utils.cpp_extension``): every ``csrc/*.hip`` file is compiled for
``--offload-arch=gfx950`` into an object file and the objects are linked into one
shared library next to this file.  ``ops/_lib.py`` loads it with ``ctypes`` after
``import torch`` so the process keeps a single HIP runtime (torch's
``libamdhip64.so.7``; the library's dependency resolves to the already-loaded
soname).

Usage::

    python -m distributed_pytorch_cookbook_amd.ops.build [--force] [-j N]
"""
from __future__ import annotations

import argparse
import os
import shutil
import subprocess
import sys
from concurrent.futures import ThreadPoolExecutor
from pathlib import Path

HERE = Path(__file__).resolve().parent
CSRC = HERE / "csrc"
BUILD_DIR = HERE / "_build"
LIB_PATH = HERE / "libdpc_kernels.so"
ARCH = os.environ.get("DPC_OFFLOAD_ARCH", "gfx950")

# gemm7_part*.hip: the persistent GEMM kernels' instantiations, dealt over several files that
# compile in parallel (ops/gen_gemm_parts.py; gemm7.hip itself is the host-side dispatcher)
SOURCES = ["gemm.hip", "gemm7.hip", "gemm_f32.hip", "attention.hip", "attention_f32.hip", "layernorm.hip", "misc.hip",
           "decode.hip", "embed_bwd.hip", "ipc_coll.hip"] + sorted(p.name for p in CSRC.glob("gemm7_part*.hip"))
HEADERS = ["common.h", "gemm.h", "gemm7_kern.h", "gemm9_kern.h", "gemm7_extern.inc"]

# code-object v5 keeps the library loadable by torch's bundled ROCm 7.0 runtime as
# well as by the 7.2 toolchain in /opt/rocm.
CFLAGS = [
    f"--offload-arch={ARCH}",
    "-O3",
    "-std=c++17",
    "-fPIC",
    "-mcode-object-version=5",
    "-ffp-contract=fast",
    "-Wno-unused-result",
]


def hipcc() -> str:
    for cand in (os.environ.get("HIPCC"), shutil.which("hipcc"), "/opt/rocm/bin/hipcc"):
        if cand and Path(cand).exists():
            return cand
    raise RuntimeError("hipcc not found: cannot build the gfx950 kernel library")


# per-file extras: attention never produces NaNs (masked scores are -inf), so maxnum needs
# no canonicalisation of MFMA results and folds into v_max3_f32
# attention.hip: -fno-slp-vectorize -- at -O3 the SLP vectoriser packed the softmax row sums
# into v_pk_add_f32 fed by v_mov_b32 pairs (32 moves + 13 packed adds per tile instead of 32
# adds) and the dS products into v_pk_mul_f32; packed f32 VALU beside MFMAs costs extra issue
# cycles (MI355X_MICROARCH.md: "an anti-lever beside MFMAs")
FILE_FLAGS = {"attention.hip": ["-fno-honor-nans", "-fno-slp-vectorize"], "attention_f32.hip": ["-fno-honor-nans"]}


HASH_PATH = LIB_PATH.with_suffix(".so.srchash")


def source_hash() -> str:
    """Content hash of the sources + flags (mtimes do not survive snapshot copies)."""
    import hashlib

    h = hashlib.sha256((" ".join(CFLAGS) + repr(sorted(FILE_FLAGS.items()))).encode())
    for name in SOURCES + HEADERS:
        h.update(name.encode())
        h.update((CSRC / name).read_bytes())
    return h.hexdigest()


def needs_build() -> bool:
    if not LIB_PATH.exists() or not HASH_PATH.exists():
        return True
    return HASH_PATH.read_text().strip() != source_hash()


def _compile(src: Path, obj: Path, verbose: bool) -> None:
    cmd = [hipcc(), *CFLAGS, *FILE_FLAGS.get(src.name, []), "-c", str(src), "-o", str(obj)]
    if verbose:
        print(" ".join(cmd), flush=True)
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"hipcc failed for {src.name}:\n{r.stdout}\n{r.stderr}")


def _deps(name: str, seen=None) -> set:
    """The local headers ``name`` includes, transitively."""
    import re

    seen = set() if seen is None else seen
    for inc in re.findall(r'^#include "([^"]+)"', (CSRC / name).read_text(), re.M):
        if inc not in seen and (CSRC / inc).exists():
            seen.add(inc)
            _deps(inc, seen)
    return seen


def _obj_hash(name: str) -> str:
    """Content hash of one object's inputs: its source, the local headers it includes
    (transitively), the compiler and the flags it is built with (CFLAGS + its FILE_FLAGS)."""
    import hashlib

    h = hashlib.sha256((" ".join(CFLAGS + FILE_FLAGS.get(name, [])) + "\0" + hipcc()).encode())
    for dep in [name] + sorted(_deps(name)):
        h.update(dep.encode() + b"\0")
        h.update((CSRC / dep).read_bytes())
    return h.hexdigest()


def build(force: bool = False, jobs: int = 8, verbose: bool = False) -> Path:
    if not force and not needs_build():
        return LIB_PATH
    BUILD_DIR.mkdir(exist_ok=True)
    todo = []
    objs = []
    for s in SOURCES:
        src, obj = CSRC / s, BUILD_DIR / (Path(s).stem + ".o")
        objs.append(obj)
        # rebuilt when the recorded input hash differs (mtimes do not survive snapshot copies, and
        # a flags-only change leaves every mtime alone)
        stamp = obj.with_suffix(".o.hash")
        want = _obj_hash(s)
        if force or not obj.exists() or not stamp.exists() or stamp.read_text().strip() != want:
            todo.append((src, obj, stamp, want))
    # the longest compiles first (the GEMM parts), so the pool's tail is short
    todo.sort(key=lambda so: 0 if "gemm7" in so[0].name else 1)

    def one(item):
        src, obj, stamp, want = item
        stamp.unlink(missing_ok=True)
        _compile(src, obj, verbose)
        stamp.write_text(want + "\n")

    with ThreadPoolExecutor(max_workers=max(1, jobs)) as ex:
        list(ex.map(one, todo))
    tmp = LIB_PATH.with_suffix(".so.tmp")
    cmd = [hipcc(), f"--offload-arch={ARCH}", "-shared", "-fPIC", *map(str, objs), "-o", str(tmp)]
    if verbose:
        print(" ".join(cmd), flush=True)
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"link failed:\n{r.stdout}\n{r.stderr}")
    os.replace(tmp, LIB_PATH)
    HASH_PATH.write_text(source_hash() + "\n")
    return LIB_PATH


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(description=__doc__)
    ap.add_argument("--force", action="store_true")
    ap.add_argument("-j", "--jobs", type=int, default=8)
    ap.add_argument("-v", "--verbose", action="store_true")
    a = ap.parse_args(argv)
    path = build(force=a.force, jobs=a.jobs, verbose=a.verbose)
    print(f"built {path}")
    return 0


if __name__ == "__main__":
    sys.exit(main())
