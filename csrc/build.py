"""Build the vgate native extension (``vgate/_C*.so``) for gfx950 in-tree.

Design: the HIP kernels (``csrc/kernels/*.hip``) are compiled by ``hipcc
--offload-arch=gfx950`` WITHOUT torch headers (fast, seconds per file); the
only torch-aware translation units are the binding/runtime ``.cpp`` files,
compiled as plain host C++. Everything is linked into one shared object that
resolves ``libamdhip64.so.7`` to the copy torch already loaded (same SONAME),
so kernels run on torch's HIP runtime and streams.

Usage: ``python csrc/build.py [--force] [-j N]``
"""
from __future__ import annotations

import argparse
import os
import subprocess
import sys
import sysconfig
from concurrent.futures import ThreadPoolExecutor
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
CSRC = ROOT / "csrc"
BUILD = ROOT / "build" / "csrc"
ARCH = os.environ.get("VGATE_OFFLOAD_ARCH", "gfx950")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")


def ext_path() -> Path:
    return ROOT / "vgate" / ("_C" + sysconfig.get_config_var("EXT_SUFFIX"))


def _torch_paths():
    import torch  # noqa: F401  (import only for its install location)
    from torch.utils import cpp_extension

    return cpp_extension.include_paths(), cpp_extension.library_paths()[0], bool(torch._C._GLIBCXX_USE_CXX11_ABI)


def _newer(src: Path, obj: Path, deps: list[Path]) -> bool:
    if not obj.exists():
        return True
    t = obj.stat().st_mtime
    return src.stat().st_mtime > t or any(d.stat().st_mtime > t for d in deps)


def _run(cmd: list[str]) -> None:
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        sys.stderr.write(" ".join(cmd) + "\n" + r.stdout + r.stderr)
        raise RuntimeError(f"compile failed: {cmd[-1]}")


def build(force: bool = False, jobs: int = 8, verbose: bool = True) -> Path:
    BUILD.mkdir(parents=True, exist_ok=True)
    incs, torch_lib, cxx11 = _torch_paths()
    py_inc = sysconfig.get_paths()["include"]
    kernel_hdrs = sorted((CSRC / "kernels").glob("*.h"))
    rt_hdrs = sorted((CSRC / "runtime").glob("*.h"))
    jobs_list = []
    common = ["-O3", "-std=c++17", "-fPIC"]
    want = []  # this tree's objects: a stale object of a deleted / renamed source is never linked
    for src in sorted((CSRC / "kernels").glob("*.hip")):
        obj = BUILD / (src.stem + ".o")
        want.append(obj)
        if force or _newer(src, obj, kernel_hdrs):
            cmd = [HIPCC, f"--offload-arch={ARCH}", *common, "-munsafe-fp-atomics",
                   "-Wno-unused-result", "-c", str(src), "-o", str(obj)]
            jobs_list.append(cmd)
    host_flags = [
        "-D__HIP_PLATFORM_AMD__=1", "-DUSE_ROCM=1", "-DTORCH_EXTENSION_NAME=_C",
        "-DTORCH_API_INCLUDE_EXTENSION_H", f"-D_GLIBCXX_USE_CXX11_ABI={int(cxx11)}",
        "-I/opt/rocm/include", f"-I{py_inc}", *[f"-I{i}" for i in incs],
        "-Wno-deprecated-declarations", "-Wno-unused-parameter",
    ]
    for src in sorted((CSRC / "runtime").glob("*.cpp")):
        obj = BUILD / (src.stem + ".o")
        want.append(obj)
        if force or _newer(src, obj, kernel_hdrs + rt_hdrs):
            jobs_list.append(["g++", *common, *host_flags, "-c", str(src), "-o", str(obj)])
    if jobs_list:
        if verbose:
            print(f"[vgate.build] compiling {len(jobs_list)} translation unit(s) for {ARCH}", flush=True)
        with ThreadPoolExecutor(max_workers=max(1, jobs)) as ex:
            list(ex.map(_run, jobs_list))
    objs = sorted(want)
    out = ext_path()
    if force or jobs_list or not out.exists() or any(o.stat().st_mtime > out.stat().st_mtime for o in objs):
        link = [HIPCC, f"--offload-arch={ARCH}", "-shared", "-fPIC", *map(str, objs), "-o", str(out),
                f"-L{torch_lib}", "-lc10", "-lc10_hip", "-ltorch", "-ltorch_cpu", "-ltorch_hip",
                "-ltorch_python", f"-Wl,-rpath,{torch_lib}"]
        _run(link)
        if verbose:
            print(f"[vgate.build] linked {out.relative_to(ROOT)}", flush=True)
    return out


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--force", action="store_true")
    ap.add_argument("-j", "--jobs", type=int, default=min(8, os.cpu_count() or 4))
    a = ap.parse_args()
    build(force=a.force, jobs=a.jobs)


if __name__ == "__main__":
    main()
