"""In-tree native build: C++ runtime core (g++) and HIP/CDNA4 kernels (hipcc, gfx950).

Both libraries are pybind11 modules written next to the package so that the
built ``.so`` travels with the repository snapshot to the GPU box:

  xgserve/_runtime*.so   <- csrc/runtime/*.cpp   (host C++17, no GPU deps)
  xgserve/_kernels*.so   <- csrc/kernels/*.hip + csrc/comm/*.hip  (hipcc --offload-arch=gfx950)

The kernel library is linked against the HIP runtime that PyTorch itself loads
(``torch/lib/libamdhip64.so``, same SONAME as /opt/rocm's), so one HIP runtime
instance serves torch and our kernels. Kernels take raw device pointers and the
current hipStream_t from Python -- no torch C++ headers, no hipify.

Usage:  python -m xgserve._build [--force] [--jobs N] [--only runtime|kernels]
"""
from __future__ import annotations

import argparse
import concurrent.futures as cf
import hashlib
import os
import subprocess
import sys
import sysconfig
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
PKG = ROOT / "xgserve"
CSRC = ROOT / "csrc"
BUILD = ROOT / "build" / "obj"
EXT = sysconfig.get_config_var("EXT_SUFFIX") or ".so"
ARCH = os.environ.get("XGS_OFFLOAD_ARCH", "gfx950")


def _pybind_includes() -> list:
    import pybind11
    return [f"-I{pybind11.get_include()}", f"-I{sysconfig.get_paths()['include']}"]


def _torch_lib() -> str:
    import importlib.util
    spec = importlib.util.find_spec("torch")
    return str(Path(spec.origin).parent / "lib")


def _digest(paths, flags) -> str:
    h = hashlib.sha256()
    for p in sorted(paths):
        h.update(str(p).encode())
        h.update(Path(p).read_bytes())
    h.update(" ".join(flags).encode())
    return h.hexdigest()[:16]


def _run(cmd):
    r = subprocess.run(cmd, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True)
    if r.returncode != 0:
        sys.stderr.write(" ".join(cmd) + "\n" + r.stdout)
        raise RuntimeError(f"build step failed: {cmd[0]} ... {cmd[-1]}")
    return r.stdout


def _needs(out: Path, stamp: str, force: bool) -> bool:
    st = out.with_suffix(out.suffix + ".stamp")
    return force or not out.exists() or not st.exists() or st.read_text() != stamp


def _write_stamp(out: Path, stamp: str):
    out.with_suffix(out.suffix + ".stamp").write_text(stamp)


def build_runtime(force: bool = False, jobs: int = 8, extra=()) -> Path:
    srcs = sorted((CSRC / "runtime").glob("*.cpp"))
    hdrs = sorted((CSRC / "runtime").glob("*.h"))
    out = PKG / f"_runtime{EXT}"
    flags = ["-O3", "-std=c++17", "-fPIC", "-Wall", "-Wno-sign-compare", "-fvisibility=hidden", *extra]
    stamp = _digest(srcs + hdrs, flags)
    if not _needs(out, stamp, force):
        return out
    obj_dir = BUILD / "runtime"
    obj_dir.mkdir(parents=True, exist_ok=True)
    inc = _pybind_includes() + [f"-I{CSRC / 'runtime'}"]

    def cc(src):
        o = obj_dir / (src.stem + ".o")
        _run(["g++", *flags, *inc, "-c", str(src), "-o", str(o)])
        return o

    with cf.ThreadPoolExecutor(max_workers=jobs) as ex:
        objs = list(ex.map(cc, srcs))
    _run(["g++", "-shared", *flags, *map(str, objs), "-o", str(out)])
    _write_stamp(out, stamp)
    return out


def build_kernels(force: bool = False, jobs: int = 8, probes: bool = False) -> Path:
    """probes: also compile the anatomy-probe kernels (gemm_pf without DMA / MFMA,
    decode attention without prologue / key loop). They are measurement builds
    (bench/pf_gemm_bench.py --probe, bench/decode_cold.py --probe), never selected
    by a plan, so the default library leaves them out."""
    srcs = sorted((CSRC / "kernels").glob("*.hip")) + sorted((CSRC / "comm").glob("*.hip"))
    hdrs = sorted((CSRC / "kernels").glob("*.h")) + sorted((CSRC / "comm").glob("*.h"))
    cpp = sorted((CSRC / "kernels").glob("*.cpp"))
    out = PKG / f"_kernels{EXT}"
    flags = ["-O3", "-std=c++17", "-fPIC", f"--offload-arch={ARCH}", "-fvisibility=hidden",
             "-munsafe-fp-atomics", "-Wno-unused-result"] + (["-DXGK_PROBES=1"] if probes else [])
    stamp = _digest(srcs + hdrs + cpp, flags)
    if not _needs(out, stamp, force):
        return out
    obj_dir = BUILD / "kernels"
    obj_dir.mkdir(parents=True, exist_ok=True)
    inc = _pybind_includes() + [f"-I{CSRC / 'kernels'}", f"-I{CSRC / 'comm'}"]

    def cc(src):
        o = obj_dir / (src.stem + ".o")
        _run(["hipcc", *flags, *inc, "-c", str(src), "-o", str(o)])
        return o

    with cf.ThreadPoolExecutor(max_workers=jobs) as ex:
        objs = list(ex.map(cc, srcs + cpp))
    tl = _torch_lib()
    _run(["hipcc", "-shared", f"--offload-arch={ARCH}", "-fPIC", *map(str, objs),
          f"-L{tl}", f"-Wl,-rpath,{tl}", "-lamdhip64", "-o", str(out)])
    _write_stamp(out, stamp)
    return out


def build_all(force: bool = False, jobs: int = 8):
    return build_runtime(force, jobs), build_kernels(force, jobs)


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--force", action="store_true")
    ap.add_argument("--jobs", type=int, default=min(8, os.cpu_count() or 4))
    ap.add_argument("--only", choices=["runtime", "kernels"], default=None)
    ap.add_argument("--probes", action="store_true", help="include the anatomy-probe kernels (measurement builds)")
    a = ap.parse_args(argv)
    if a.only in (None, "runtime"):
        print("runtime:", build_runtime(a.force, a.jobs))
    if a.only in (None, "kernels"):
        print("kernels:", build_kernels(a.force, a.jobs, a.probes))


if __name__ == "__main__":
    main()
