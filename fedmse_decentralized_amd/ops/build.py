"""In-tree build of the native libraries.

* ``libfedmx_host.so`` – C++17 host runtime (CSV reader, exact AUC); built
  with g++, needs no GPU toolchain.
* ``libfedmx_hip.so``  – hand-written CDNA4 kernels for gfx950, built with
  ``hipcc --offload-arch=gfx950``; a plain C ABI loaded with ctypes (no torch
  headers, so a rebuild takes seconds, not minutes).

Both land in ``fedmse_decentralized_amd/ops/lib/`` so they travel with the
repository snapshot to the GPU box.  ``python -m fedmse_decentralized_amd.ops.build``
rebuilds what is stale.

Staleness is decided by content, not by file times: every library has a
``<lib>.buildhash`` stamp next to it holding the SHA-256 of its compiler,
flags and the bytes of every source and header that goes into it.  A library
whose stamp is missing or differs is rebuilt (a copied tree with fresh mtimes
rebuilds nothing; an edited source is never hidden by a newer ``.so``).
"""
from __future__ import annotations

import hashlib
import os
import shutil
import subprocess
import sys
from pathlib import Path

HERE = Path(__file__).resolve().parent
CSRC = HERE / "csrc"
LIBDIR = HERE / "lib"
HOST_LIB = LIBDIR / "libfedmx_host.so"
HIP_LIB = LIBDIR / "libfedmx_hip.so"
HIP_STAMPS_LIB = LIBDIR / "libfedmx_hip_stamps.so"
OFFLOAD_ARCH = os.environ.get("FEDMX_OFFLOAD_ARCH", "gfx950")


def _sources(sub: str, exts):
    d = CSRC / sub
    return sorted(p for p in d.iterdir() if p.suffix in exts)


def _headers():
    return sorted(p for p in CSRC.rglob("*") if p.suffix in (".h", ".hpp", ".cuh", ".inc"))


def _hash_path(target: Path) -> Path:
    return target.with_name(target.name + ".buildhash")


def content_hash(cmd, deps) -> str:
    """SHA-256 over the compile command (sans output path) and every input's
    name and bytes, in a fixed order."""
    h = hashlib.sha256()
    h.update("\0".join(map(str, cmd)).encode())
    for p in sorted(set(deps), key=lambda q: q.relative_to(CSRC).as_posix()):
        h.update(b"\0" + p.relative_to(CSRC).as_posix().encode() + b"\0")
        h.update(p.read_bytes())
    return h.hexdigest()


def _stale(target: Path, digest: str) -> bool:
    hp = _hash_path(target)
    if not target.exists() or not hp.exists():
        return True
    return hp.read_text().strip() != digest


def _stamp(target: Path, digest: str) -> None:
    _hash_path(target).write_text(digest + "\n")


def _run(cmd, cwd=None):
    r = subprocess.run(cmd, cwd=cwd, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True)
    if r.returncode != 0:
        raise RuntimeError("build failed: " + " ".join(map(str, cmd)) + "\n" + r.stdout)
    return r.stdout


def build_host(force: bool = False, verbose: bool = False) -> Path:
    srcs = _sources("host", (".cpp",))
    cxx = os.environ.get("CXX", "g++")
    flags = [cxx, "-std=c++17", "-O3", "-fPIC", "-shared", "-pthread", "-Wall"]
    digest = content_hash(flags + [p.name for p in srcs], srcs + _headers())
    if not force and not _stale(HOST_LIB, digest):
        return HOST_LIB
    LIBDIR.mkdir(parents=True, exist_ok=True)
    tmp = HOST_LIB.with_suffix(".so.tmp")
    cmd = flags + [*map(str, srcs), "-o", str(tmp)]
    out = _run(cmd)
    os.replace(tmp, HOST_LIB)
    _stamp(HOST_LIB, digest)
    if verbose:
        print(out, end="")
    return HOST_LIB


def hipcc_path() -> str:
    p = shutil.which("hipcc") or "/opt/rocm/bin/hipcc"
    if not Path(p).exists():
        raise RuntimeError("hipcc not found (ROCm toolchain required to build libfedmx_hip.so)")
    return p


def build_hip(force: bool = False, verbose: bool = False, extra_flags=(), target: Path = HIP_LIB) -> Path:
    """``extra_flags``/``target`` build variants next to the main library, e.g.
    the in-kernel timestamp build ``-DFEDMX_STAMPS=1`` -> ``libfedmx_hip_stamps.so``
    (selected at load time with ``FEDMX_HIP_LIB``)."""
    srcs = _sources("hip", (".hip",))
    # -ffp-contract=off: separately rounded mul/add like the torch ops the kernels
    # reproduce (aggregation sums are then bit-identical to the reference order)
    # -amdgpu-mfma-vgpr-form: MFMA accumulators in arch VGPRs (the training
    # kernel otherwise pays ~150 v_accvgpr moves per step on its VALU-bound
    # optimizer tail: -3.3% launch time measured)
    flags = [f"--offload-arch={OFFLOAD_ARCH}", "-O3", "-std=c++17", "-fPIC", "-shared",
             "-ffp-contract=off", "-munsafe-fp-atomics", "-mllvm", "-amdgpu-mfma-vgpr-form=1", *extra_flags]
    digest = content_hash(["hipcc", *flags, *(p.name for p in srcs)], srcs + _headers())
    if not force and not _stale(target, digest):
        return target
    LIBDIR.mkdir(parents=True, exist_ok=True)
    tmp = target.with_suffix(".so.tmp")
    cmd = [hipcc_path(), *flags, f"-I{CSRC / 'hip'}", *map(str, srcs), "-o", str(tmp)]
    out = _run(cmd)
    os.replace(tmp, target)
    _stamp(target, digest)
    if verbose:
        print(out, end="")
    return target


def build_all(force: bool = False, verbose: bool = False):
    return build_host(force, verbose), build_hip(force, verbose)


if __name__ == "__main__":
    force = "--force" in sys.argv
    for p in build_all(force=force, verbose=True):
        print("built", p)
