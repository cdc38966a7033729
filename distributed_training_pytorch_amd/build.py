"""Build the native library ``_lib/libdtp.so`` with hipcc for gfx950.

Every ``csrc/*.hip`` file is compiled separately (``hipcc -c``, parallel) and
linked into one shared object with a plain C ABI, loaded through ctypes by
``_native.py``.  Built in-tree so the ``.so`` travels with the repository
snapshot to the GPU box.  No hipify, no CUDA sources: the kernels are written
for CDNA4 directly.
"""
from __future__ import annotations

import concurrent.futures as cf
import hashlib
import os
import shutil
import subprocess
import sys
from pathlib import Path

PKG = Path(__file__).resolve().parent
CSRC = PKG / "csrc"
LIBDIR = PKG / "_lib"
OBJDIR = LIBDIR / "obj"
LIB = LIBDIR / "libdtp.so"
ARCH = os.environ.get("DTP_OFFLOAD_ARCH", "gfx950")

COMMON_FLAGS = [
    "-O3",
    "-std=c++17",
    "-fPIC",
    f"--offload-arch={ARCH}",
    "-mcode-object-version=5",
    "-Wno-unused-result",
    "-Wno-unused-command-line-argument",
]


# per-source flags: the fused step runs one wave per SIMD, nothing hides its
# latencies but its own ILP -> the max-ILP machine scheduler (measured 4.83-4.91
# vs 5.08 us/step with the default occupancy-driven one, docs/perf_notes.md)
# -ffp-contract=off where the optimizer math lives: every fused multiply-add there is
# an explicit fmaf, so kernel instances scheduled differently round identically
SOURCE_FLAGS = {"mlp_train.hip": ["-mllvm", "-amdgpu-sched-strategy=max-ilp", "-ffp-contract=off"],
                "optim.hip": ["-ffp-contract=off"],
                "split_train.hip": ["-mllvm", "-amdgpu-sched-strategy=max-ilp", "-ffp-contract=off"]}


def hipcc() -> str:
    for cand in (os.environ.get("HIPCC"), shutil.which("hipcc"), "/opt/rocm/bin/hipcc"):
        if cand and Path(cand).exists():
            return cand
    raise RuntimeError("hipcc not found: install ROCm or set HIPCC")


def _sources() -> list[Path]:
    return sorted(CSRC.glob("*.hip"))


def _headers() -> list[Path]:
    return sorted(CSRC.glob("*.h"))


def source_hash() -> str:
    """sha256 (16 hex) over every csrc source and header and the compile flags: the
    identity of a build.  ``runtime.hip`` bakes it into the library
    (``dtp_source_hash()``) and ``_native.load()`` refuses a library whose stamp is
    not the hash of the sources next to it -- so the kernel that ran is tied to the
    sources of the commit, not to file modification times."""
    h = hashlib.sha256()
    for f in sorted([*CSRC.glob("*.hip"), *CSRC.glob("*.h")]):
        h.update(f.name.encode())
        h.update(b"\0")
        h.update(f.read_bytes())
    h.update(repr((COMMON_FLAGS, sorted(SOURCE_FLAGS.items()))).encode())
    return h.hexdigest()[:16]


def _stamp_ok(target: Path, stamp: str) -> bool:
    sf = target.with_name(target.name + ".sha")
    return target.exists() and sf.exists() and sf.read_text().strip() == stamp


def _write_stamp(target: Path, stamp: str) -> None:
    target.with_name(target.name + ".sha").write_text(stamp + "\n")


def _obj_stamp(src: Path, full: str) -> str:
    """An object depends on its source, every header (cheap to over-approximate) and
    the flags; runtime.hip also on the whole-tree hash it embeds."""
    h = hashlib.sha256(src.read_bytes())
    for f in _headers():
        h.update(f.read_bytes())
    h.update(repr((COMMON_FLAGS, SOURCE_FLAGS.get(src.name))).encode())
    if src.name == "runtime.hip":
        h.update(full.encode())
    return h.hexdigest()[:16]


def _extra_flags(src: Path, full: str) -> list[str]:
    return [f'-DDTP_SOURCE_HASH="{full}"'] if src.name == "runtime.hip" else []


def _compile(src: Path, verbose: bool, full: str) -> Path:
    obj = OBJDIR / (src.stem + ".o")
    stamp = _obj_stamp(src, full)
    if _stamp_ok(obj, stamp):
        return obj
    cmd = [hipcc(), *COMMON_FLAGS, *SOURCE_FLAGS.get(src.name, []), *_extra_flags(src, full), "-I", str(CSRC), "-c",
           str(src), "-o", str(obj)]
    if verbose:
        print(" ".join(cmd), flush=True)
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"hipcc failed for {src.name}:\n{r.stdout}\n{r.stderr}")
    _write_stamp(obj, stamp)
    return obj


def variant(name: str, flags: list[str], sources: tuple[str, ...] = ("mlp_train.hip",),
            verbose: bool = False) -> Path:
    """A/B build: ``sources`` recompiled with extra ``flags`` (e.g. ``-DDTP_BWD_PK=0``)
    into ``_lib/var_<name>/libdtp.so``, linked with the default objects of every other
    source.  Load it with ``DTP_LIB=<path>`` (``_native.LIB_PATH``)."""
    build(verbose=verbose)
    vdir = LIBDIR / f"var_{name}"
    (vdir / "obj").mkdir(parents=True, exist_ok=True)
    objs = []
    for src in _sources():
        if src.name in sources:
            obj = vdir / "obj" / (src.stem + ".o")
            cmd = [hipcc(), *COMMON_FLAGS, *SOURCE_FLAGS.get(src.name, []), *_extra_flags(src, source_hash()),
                   *flags, "-I", str(CSRC), "-c", str(src), "-o", str(obj)]
            if verbose:
                print(" ".join(cmd), flush=True)
            r = subprocess.run(cmd, capture_output=True, text=True)
            if r.returncode != 0:
                raise RuntimeError(f"hipcc failed for {src.name} ({name}):\n{r.stdout}\n{r.stderr}")
            objs.append(obj)
        else:
            objs.append(OBJDIR / (src.stem + ".o"))
    lib = vdir / "libdtp.so"
    r = subprocess.run([hipcc(), "-shared", "-fPIC", f"--offload-arch={ARCH}", "-o", str(lib), *map(str, objs)],
                       capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"link failed ({name}):\n{r.stdout}\n{r.stderr}")
    return lib


def build(verbose: bool = False, jobs: int | None = None) -> Path:
    """Compile (incrementally) and link libdtp.so; returns its path."""
    OBJDIR.mkdir(parents=True, exist_ok=True)
    srcs = _sources()
    jobs = jobs or min(len(srcs), max(1, (os.cpu_count() or 4) // 2), 8)
    full = source_hash()
    with cf.ThreadPoolExecutor(max_workers=jobs) as ex:
        objs = list(ex.map(lambda s: _compile(s, verbose, full), srcs))
    if not _stamp_ok(LIB, full):
        tmp = LIB.with_suffix(".so.tmp")
        cmd = [hipcc(), "-shared", "-fPIC", f"--offload-arch={ARCH}", "-o", str(tmp), *map(str, objs)]
        if verbose:
            print(" ".join(cmd), flush=True)
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError(f"link failed:\n{r.stdout}\n{r.stderr}")
        os.replace(tmp, LIB)
        _write_stamp(LIB, full)
    return LIB


def asm(src_name: str, out_dir: Path | None = None) -> Path:
    """Emit the device assembly (.s) of one source for inspection."""
    out_dir = out_dir or (LIBDIR / "asm")
    out_dir.mkdir(parents=True, exist_ok=True)
    src = CSRC / src_name
    cmd = [hipcc(), *COMMON_FLAGS, *SOURCE_FLAGS.get(src.name, []), "-I", str(CSRC), "--cuda-device-only", "-S", str(src),
           "-o", str(out_dir / (src.stem + ".s"))]
    subprocess.run(cmd, check=True)
    return out_dir / (src.stem + ".s")


if __name__ == "__main__":
    # python -m distributed_training_pytorch_amd.build [-v] [--variant NAME [--sources a.hip,b.hip] FLAG...]
    if "--variant" in sys.argv:
        i = sys.argv.index("--variant")
        rest = [x for x in sys.argv[i + 2:] if x != "-v"]
        srcs = ("mlp_train.hip",)
        if "--sources" in rest:
            j = rest.index("--sources")
            srcs = tuple(rest[j + 1].split(","))
            rest = rest[:j] + rest[j + 2:]
        print(variant(sys.argv[i + 1], rest, srcs, verbose="-v" in sys.argv))
    else:
        print(build(verbose="-v" in sys.argv))
