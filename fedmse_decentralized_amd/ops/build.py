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
``<lib>.buildhash`` stamp next to it holding the SHA-256 of its compiler's
identity (resolved path + ``--version`` output), flags and the bytes of every
source and header that goes into it.  A library whose stamp is missing or
differs is rebuilt (a copied tree with fresh mtimes rebuilds nothing; an
edited source is never hidden by a newer ``.so``; a different toolchain on
the machine that imports the tree rebuilds).  ``BUILD_STATUS`` records, per
library, whether this process compiled it or reused it and under which hash.
"""
from __future__ import annotations

import functools
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
# IEEE-division Adam variant (-DFEDMX_EXACT_ADAM=1): long-horizon parity test
HIP_EXACT_LIB = LIBDIR / "libfedmx_hip_exact.so"
OFFLOAD_ARCH = os.environ.get("FEDMX_OFFLOAD_ARCH", "gfx950")

# target path -> (action "compiled" | "reused", content hash) for this process
BUILD_STATUS: dict = {}


@functools.lru_cache(maxsize=None)
def compiler_identity(exe: str) -> str:
    """Resolved path and ``--version`` banner of a compiler: part of every
    build hash, so a library built by another toolchain counts as stale."""
    path = shutil.which(exe) or exe
    real = os.path.realpath(path)
    try:
        r = subprocess.run([real, "--version"], stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True,
                           timeout=60)
        ver = r.stdout.strip()
    except (OSError, subprocess.SubprocessError) as e:
        ver = f"unavailable: {e}"
    return f"{real}\n{ver}"


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
    """Run one command (a list of arguments) or several in order (a list of such lists)."""
    if cmd and isinstance(cmd[0], (list, tuple)):
        return "".join(_run(c, cwd) for c in cmd)
    r = subprocess.run(cmd, cwd=cwd, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True)
    if r.returncode != 0:
        raise RuntimeError("build failed: " + " ".join(map(str, cmd)) + "\n" + r.stdout)
    return r.stdout


def _build(target: Path, digest: str, cmd_for, force: bool, verbose: bool) -> Path:
    """Compile ``target`` unless its stamp already matches ``digest``.  The
    check-and-compile runs under an exclusive lock on ``<lib>.lock``, so ranks
    or tests that import a stale tree at once compile it once; the others
    find it fresh and reuse it.  ``cmd_for(tmp)`` gives the compile command
    writing to a per-process temporary file, renamed into place atomically."""
    if not force and not _stale(target, digest):
        BUILD_STATUS[target] = ("reused", digest)
        return target
    import fcntl

    target.parent.mkdir(parents=True, exist_ok=True)
    with open(target.with_name(target.name + ".lock"), "w") as lk:
        fcntl.flock(lk, fcntl.LOCK_EX)
        if not force and not _stale(target, digest):   # another process built it meanwhile
            BUILD_STATUS[target] = ("reused", digest)
            return target
        tmp = target.with_name(f"{target.name}.{os.getpid()}.tmp")
        try:
            out = _run(cmd_for(tmp))
        finally:
            for o in target.parent.glob(f"{tmp.name}.*.o"):   # per-source objects (hip_link_commands)
                o.unlink()
        os.replace(tmp, target)
        _stamp(target, digest)
    BUILD_STATUS[target] = ("compiled", digest)
    if verbose:
        print(out, end="")
    return target


def build_host(force: bool = False, verbose: bool = False) -> Path:
    srcs = _sources("host", (".cpp",))
    cxx = os.environ.get("CXX", "g++")
    flags = [cxx, "-std=c++17", "-O3", "-fPIC", "-shared", "-pthread", "-Wall"]
    digest = content_hash([compiler_identity(cxx)] + flags + [p.name for p in srcs], srcs + _headers())
    return _build(HOST_LIB, digest, lambda tmp: flags + [*map(str, srcs), "-o", str(tmp)], force, verbose)


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
    base = _hip_flags(extra_flags)
    flags = [*base[:3], "-fPIC", "-shared", *base[3:]]
    digest = content_hash([compiler_identity(hipcc_path()), *flags, *(p.name for p in srcs),
                           *(f"{k}:{' '.join(v)}" for k, v in sorted(SOURCE_FLAGS.items()))], srcs + _headers())
    return _build(target, digest, lambda tmp: hip_link_commands(srcs, flags, CSRC / "hip", tmp), force, verbose)


# Per-source flags, added to the library's for that translation unit only: the
# FedProx instantiation of the helper-wave training kernel compiles with the
# machine scheduler's memory-operation clustering off (966 -> 939 us per
# launch; the same flag costs the other instantiations 1-2.5 %,
# profiles/r6_fedprox_nocluster.md)
SOURCE_FLAGS = {"fedmx_train_hw_prox.hip": ["-mllvm", "-misched-cluster=false"]}


def hip_link_commands(srcs, flags, include_dir: Path, out: Path) -> list:
    """The commands that build one kernel library: every source listed in
    SOURCE_FLAGS compiled to an object of its own (``<out>.<stem>.o``), then
    one hipcc line over the other sources and those objects."""
    cmds, objs, rest = [], [], []
    obj_flags = [f for f in flags if f != "-shared"]
    for p in srcs:
        extra = SOURCE_FLAGS.get(Path(p).name)
        if extra:
            o = Path(out).with_name(f"{Path(out).name}.{Path(p).stem}.o")
            cmds.append([hipcc_path(), *obj_flags, *extra, f"-I{include_dir}", "-c", str(p), "-o", str(o)])
            objs.append(o)
        else:
            rest.append(p)
    # (objects before the sources: hipcc marks every source `-x hip`, which would also apply to a later object)
    cmds.append([hipcc_path(), *flags, f"-I{include_dir}", *map(str, objs), *map(str, rest), "-o", str(out)])
    return cmds


def _hip_flags(extra_flags=()):
    return [f"--offload-arch={OFFLOAD_ARCH}", "-O3", "-std=c++17", "-ffp-contract=off", "-munsafe-fp-atomics",
            "-mllvm", "-amdgpu-mfma-vgpr-form=1", *extra_flags]


def kernel_resources(source: str = "fedmx_train_hw.hip", extra_flags=(), asm: bool = False) -> dict:
    """Per-kernel register / spill / scratch figures of one HIP source as the
    library's flags compile it for the GPU (hipcc ``-Rpass-analysis=
    kernel-resource-usage``; no GPU needed).  Returns ``{mangled name: {"vgpr",
    "agpr", "sgpr", "vgpr_spill", "sgpr_spill", "scratch", "lds", "occupancy"}}``;
    with ``asm=True`` also ``{"__asm__": the device assembly}``."""
    import re
    import tempfile

    src = CSRC / "hip" / source
    keys = {"VGPRs": "vgpr", "AGPRs": "agpr", "TotalSGPRs": "sgpr", "VGPRs Spill": "vgpr_spill",
            "SGPRs Spill": "sgpr_spill", "ScratchSize [bytes/lane]": "scratch", "LDS Size [bytes/block]": "lds",
            "Occupancy [waves/SIMD]": "occupancy"}
    with tempfile.TemporaryDirectory() as td:
        out = Path(td) / ("k.s" if asm else "k.o")
        cmd = [hipcc_path(), *[f for f in _hip_flags(extra_flags) if f not in ("-fPIC",)], "--cuda-device-only",
               "-S" if asm else "-c", f"-I{CSRC / 'hip'}", str(src), "-o", str(out),
               "-Rpass-analysis=kernel-resource-usage"]
        log = _run(cmd)
        res: dict = {}
        cur = None
        for line in log.splitlines():
            m = re.search(r"remark:\s+(.*?) \[-Rpass-analysis", line)
            if not m:
                continue
            text = m.group(1)
            if text.startswith("Function Name:"):
                cur = res.setdefault(text.split(":", 1)[1].strip(), {})
                continue
            k, _, v = text.rpartition(":")
            if cur is not None and k.strip() in keys:
                cur[keys[k.strip()]] = int(v.strip())
        if asm:
            res["__asm__"] = out.read_text()
    return res


def train_resource_report(extra_flags=()) -> str:
    """One line per helper-wave training instantiation: VGPRs, spills, scratch."""
    names = {"_ZN5fedmx2hw15train_kernel_hwILb0ELb0EEEvNS_9TrainArgsE": "plain (batch <= 12)",
             "_ZN5fedmx2hw15train_kernel_hwILb1ELb0EEEvNS_9TrainArgsE": "FedProx (batch <= 12)",
             "_ZN5fedmx2hw15train_kernel_hwILb0ELb1EEEvNS_9TrainArgsE": "plain, batch > 12",
             "_ZN5fedmx2hw15train_kernel_hwILb1ELb1EEEvNS_9TrainArgsE": "FedProx, batch > 12"}
    res = kernel_resources("fedmx_train_hw.hip", extra_flags)
    res.update(kernel_resources("fedmx_train_hw_prox.hip", [*extra_flags, *SOURCE_FLAGS["fedmx_train_hw_prox.hip"]]))
    rows = ["instantiation            VGPR  VGPR-spill  SGPR-spill  scratch B/lane  LDS B"]
    for k, label in names.items():
        r = res.get(k, {})
        rows.append(f"{label:24s} {r.get('vgpr', '?'):>4}  {r.get('vgpr_spill', '?'):>10}  {r.get('sgpr_spill', '?'):>10}"
                    f"  {r.get('scratch', '?'):>14}  {r.get('lds', '?'):>5}")
    return "\n".join(rows)


def build_all(force: bool = False, verbose: bool = False):
    """The host runtime, the kernel library, and its IEEE-Adam variant (loaded
    only by tests/test_long_horizon_gpu.py through FEDMX_HIP_LIB)."""
    out = build_host(force, verbose), build_hip(force, verbose)
    build_hip(force, verbose, extra_flags=["-DFEDMX_EXACT_ADAM=1"], target=HIP_EXACT_LIB)
    return out


def describe(target: Path) -> str:
    """``compiled <lib> (hash …)`` or ``reused <lib> (hash …)`` for a library
    this process built or checked."""
    act, digest = BUILD_STATUS.get(target, ("not built", ""))
    return f"{act} {target} (hash {digest[:16]})" if digest else f"{act} {target}"


if __name__ == "__main__":
    if "--resources" in sys.argv:   # register / spill / scratch report of the training kernel
        print(train_resource_report())
        sys.exit(0)
    force = "--force" in sys.argv
    for p in build_all(force=force, verbose=True):
        print(describe(p))
