"""In-tree build of the native extension ``docker_dist_nn_amd._native`` for gfx950.

Device code (``csrc/kernels/*.hip``) is compiled by ``hipcc --offload-arch=gfx950``; host-only
runtime code (``csrc/runtime/*.cpp``, ``csrc/bindings.cpp``) by the host compiler against the HIP
headers, which is what allows host-side sanitizer builds (``sanitize=True``: ASan/UBSan on the
host objects only, GPU code untouched -- GPU ASan / xnack+ is not available on the pool).
The result is one shared object placed next to this file, so it travels with the repository
snapshot to the GPU box and is what the driver sees loaded.

The product build links NO vendor GEMM library: the library-GEMM entry points come from
``csrc/runtime/blaslt_stub.cpp`` (unavailable). ``--blas`` makes the comparison build instead:
``csrc/compare/blaslt.cpp`` + ``-lhipblaslt`` (hipBLASLt A/B runs, bench/gemm_vs_blas.py); it
replaces the in-tree module until the next product build.

Usage: ``python -m docker_dist_nn_amd._build [--force] [--jobs N] [--sanitize] [--blas]``.
"""
from __future__ import annotations

import argparse
import concurrent.futures as cf
import hashlib
import os
import shutil
import subprocess
import sys
import sysconfig
from pathlib import Path

PKG_DIR = Path(__file__).resolve().parent
ROOT = PKG_DIR.parent
CSRC = ROOT / "csrc"
ROCM = Path(os.environ.get("ROCM_PATH", "/opt/rocm"))
ARCH = "gfx950"
EXT_NAME = "_native" + (sysconfig.get_config_var("EXT_SUFFIX") or ".so")


def _hipcc() -> str:
    p = ROCM / "bin" / "hipcc"
    return str(p) if p.exists() else "hipcc"


def _host_cxx() -> str:
    for c in (os.environ.get("CXX"), "g++", "clang++"):
        if c and shutil.which(c):
            return c
    return _hipcc()


def _pybind_includes() -> list[str]:
    import pybind11

    inc = [f"-I{pybind11.get_include()}", f"-I{sysconfig.get_paths()['include']}"]
    return inc


def _sources(blas: bool = False) -> tuple[list[Path], list[Path]]:
    dev = sorted((CSRC / "kernels").glob("*.hip"))
    host = sorted((CSRC / "runtime").glob("*.cpp")) + [CSRC / "bindings.cpp"]
    if blas:  # comparison build: the real hipBLASLt path instead of the stub
        host = [h for h in host if h.name != "blaslt_stub.cpp"] + [CSRC / "compare" / "blaslt.cpp"]
    return dev, host


def _header_digest() -> str:
    h = hashlib.sha1()
    for p in sorted(CSRC.rglob("*.hpp")) + sorted(CSRC.rglob("*.h")):
        h.update(p.read_bytes())
    return h.hexdigest()[:12]


def _flags(sanitize: bool) -> tuple[list[str], list[str]]:
    common = ["-O3", "-std=c++17", "-fPIC", f"-I{CSRC}", "-Wall", "-Wno-unused-function"]
    # DNN_HIP_DEFINES: extra device-compile defines for A/B experiments (e.g.
    # "-DDNN_GEMM_SETPRIO=1"); they are part of the object-directory tag below
    dev = [_hipcc(), f"--offload-arch={ARCH}", *common, "-Wno-unused-result",
           *os.environ.get("DNN_HIP_DEFINES", "").split()]
    host = [_host_cxx(), *common, f"-I{ROCM / 'include'}", "-D__HIP_PLATFORM_AMD__",
            *_pybind_includes(), "-fvisibility=hidden"]
    if sanitize:
        host += ["-fsanitize=address,undefined", "-fno-omit-frame-pointer", "-O1", "-g"]
    return dev, host


def _file_flags(src: Path) -> list[str]:
    """Per-file compiler flags from a ``// build-flags: ...`` line in the first 40 lines (e.g.
    mlp_tail.hip turns off SLP vectorisation, which splits DPP row sums into mov + packed add)."""
    with open(src, encoding="utf-8") as f:
        for _, line in zip(range(40), f):
            if line.startswith("// build-flags:"):
                return line.split(":", 1)[1].split()
    return []


def _compile(cmd: list[str]) -> tuple[list[str], int, str]:
    r = subprocess.run(cmd, capture_output=True, text=True)
    return cmd, r.returncode, r.stdout + r.stderr


def build(force: bool = False, jobs: int | None = None, sanitize: bool = False,
          verbose: bool = False, blas: bool = False) -> Path:
    """Compile (incrementally) and link the extension; returns the path of the .so."""
    dev_src, host_src = _sources(blas)
    tag = "asan" if sanitize else "rel"  # (stub and library objects have distinct names)
    extra = os.environ.get("DNN_HIP_DEFINES", "")
    if extra:
        tag += "-" + hashlib.sha1(extra.encode()).hexdigest()[:8]
    obj_dir = ROOT / "build" / f"native-{tag}-{_header_digest()}"
    obj_dir.mkdir(parents=True, exist_ok=True)
    dev_cmd, host_cmd = _flags(sanitize)
    out = PKG_DIR / (EXT_NAME if not sanitize else "_native_asan.so")

    jobs_to_run, objs = [], []
    for src in dev_src + host_src:
        obj = obj_dir / (src.relative_to(CSRC).as_posix().replace("/", "__") + ".o")
        objs.append(obj)
        if force or not obj.exists() or obj.stat().st_mtime < src.stat().st_mtime:
            base = dev_cmd if src.suffix == ".hip" else host_cmd
            jobs_to_run.append([*base, *_file_flags(src), "-c", str(src), "-o", str(obj)])

    if jobs_to_run:
        n = jobs or min(8, os.cpu_count() or 4)
        with cf.ThreadPoolExecutor(max_workers=n) as ex:
            for cmd, rc, log in ex.map(_compile, jobs_to_run):
                if verbose or rc:
                    sys.stderr.write(" ".join(cmd) + "\n" + log)
                if rc:
                    raise RuntimeError(f"native build failed compiling {cmd[-3]}")

    newest = max(o.stat().st_mtime for o in objs)
    # the .so records which object set it was linked from: switching back to an older header
    # set (its objects exist and are OLDER than the .so) must still relink
    stamp = out.with_suffix(".objset")
    objset = obj_dir.name + ("+blas" if blas else "")
    stale_set = not stamp.exists() or stamp.read_text().strip() != objset
    if force or jobs_to_run or stale_set or not out.exists() or out.stat().st_mtime < newest:
        link = [_hipcc(), f"--offload-arch={ARCH}", "-shared", "-fPIC", "-o", str(out),
                *map(str, objs), f"-L{ROCM / 'lib'}", "-lamdhip64",
                *(["-lhipblaslt"] if blas else [])]
        if sanitize:
            link += ["-fsanitize=address,undefined"]
        cmd, rc, log = _compile(link)
        if verbose or rc:
            sys.stderr.write(" ".join(cmd) + "\n" + log)
        if rc:
            raise RuntimeError("native link failed")
        stamp.write_text(objset + "\n")
    return out


def main(argv: list[str] | None = None) -> int:
    ap = argparse.ArgumentParser(description=__doc__.splitlines()[0])
    ap.add_argument("--force", action="store_true")
    ap.add_argument("--jobs", type=int, default=None)
    ap.add_argument("--sanitize", action="store_true")
    ap.add_argument("-v", "--verbose", action="store_true")
    ap.add_argument("--blas", action="store_true",
                    help="comparison build: link hipBLASLt (library GEMM A/B runs only)")
    a = ap.parse_args(argv)
    p = build(force=a.force, jobs=a.jobs, sanitize=a.sanitize, verbose=a.verbose, blas=a.blas)
    print(p)
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
