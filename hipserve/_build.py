"""In-tree build of the gfx950 kernel library (``hipserve/_C.so``) and the native
CPU runtime (``hipserve/_runtime.so``).

No hipify, no JIT cache: every ``csrc/kernels/*.hip`` is compiled by ``hipcc
--offload-arch=gfx950`` into an object, the torch operator registrations are
compiled as host C++, and everything is linked into one shared object that
``torch.ops.load_library`` loads. The built ``.so`` files live next to the Python
sources, so they travel with the repo snapshot to the GPU box.

Usage: ``python -m hipserve._build [--force] [-j N] [--sanitize thread|address]``
"""
from __future__ import annotations

import argparse
import concurrent.futures as cf
import glob
import hashlib
import os
import shutil
import subprocess
import sys
import sysconfig

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "csrc")
BUILD = os.path.join(ROOT, "build", "hipserve")
PKG = os.path.join(ROOT, "hipserve")
ARCH = os.environ.get("PYTORCH_ROCM_ARCH", "gfx950")
ROCM = os.environ.get("ROCM_PATH", "/opt/rocm")
HIPCC = os.path.join(ROCM, "bin", "hipcc")

HIP_FLAGS = [
    "-O3", "-std=c++17", "-fPIC", f"--offload-arch={ARCH}",
    "-munsafe-fp-atomics", "-ffp-contract=fast", "-Wno-unused-result",
    "-Wno-unused-variable",
]


def _torch_paths():
    import torch.utils.cpp_extension as ce
    import torch

    inc = ce.include_paths()
    lib = ce.library_paths()[0]
    abi = int(torch._C._GLIBCXX_USE_CXX11_ABI)
    return inc, lib, abi


def _headers():
    return sorted(glob.glob(os.path.join(CSRC, "include", "**", "*.h"), recursive=True))


def _stamp(paths, flags):
    h = hashlib.sha1()
    for p in paths:
        with open(p, "rb") as f:
            h.update(f.read())
    h.update(" ".join(flags).encode())
    return h.hexdigest()


def _needs(obj, deps, flags):
    stamp = obj + ".stamp"
    want = _stamp(deps, flags)
    if os.path.exists(obj) and os.path.exists(stamp):
        with open(stamp) as f:
            if f.read() == want:
                return None
    return want


def _run(cmd):
    r = subprocess.run(cmd, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True)
    if r.returncode != 0:
        raise RuntimeError("build failed:\n" + " ".join(cmd) + "\n" + r.stdout)
    return r.stdout


def _compile(src, obj, cmd, want):
    out = _run(cmd)
    with open(obj + ".stamp", "w") as f:
        f.write(want)
    return src, out


def build_kernels(force: bool = False, jobs: int = 8, verbose: bool = False) -> str:
    """Build hipserve/_C.so (gfx950 kernels + torch op registrations)."""
    if not os.path.exists(HIPCC):
        raise RuntimeError(f"hipcc not found at {HIPCC}")
    os.makedirs(BUILD, exist_ok=True)
    inc, libdir, abi = _torch_paths()
    hdrs = _headers()
    inc_flags = ["-I", os.path.join(CSRC, "include")]
    tasks = []
    objs = []
    for src in sorted(glob.glob(os.path.join(CSRC, "kernels", "*.hip"))):
        obj = os.path.join(BUILD, os.path.basename(src) + ".o")
        flags = HIP_FLAGS + inc_flags
        want = _stamp([src] + hdrs, flags)
        objs.append(obj)
        if force or _needs(obj, [src] + hdrs, flags):
            tasks.append((src, obj, [HIPCC, *flags, "-c", src, "-o", obj], want))
    # host-only translation unit with the torch registrations
    bsrc = os.path.join(CSRC, "torch_bindings.cpp")
    bobj = os.path.join(BUILD, "torch_bindings.o")
    bflags = ["-O2", "-std=c++17", "-fPIC", "-D__HIP_PLATFORM_AMD__", "-DUSE_ROCM",
              f"-D_GLIBCXX_USE_CXX11_ABI={abi}", "-I", os.path.join(ROCM, "include"),
              *inc_flags] + [x for p in inc for x in ("-isystem", p)]
    want = _stamp([bsrc] + hdrs, bflags)
    objs.append(bobj)
    if force or _needs(bobj, [bsrc] + hdrs, bflags):
        tasks.append((bsrc, bobj, ["g++", *bflags, "-c", bsrc, "-o", bobj], want))
    if tasks:
        with cf.ThreadPoolExecutor(max_workers=max(1, jobs)) as ex:
            futs = [ex.submit(_compile, *t) for t in tasks]
            for f in cf.as_completed(futs):
                src, out = f.result()
                if verbose:
                    print(f"[hipserve build] {os.path.relpath(src, ROOT)}", flush=True)
                    if out.strip():
                        print(out, flush=True)
    so = os.path.join(PKG, "_C.so")
    if tasks or not os.path.exists(so):
        # Link with the host toolchain and WITHOUT -lamdhip64: the HIP runtime
        # symbols resolve through libtorch_hip's own libamdhip64, so the process
        # never maps a second (system) HIP runtime next to torch's.
        link = ["g++", "-shared", "-fPIC", "-o", so + ".tmp", *objs,
                "-L", libdir, "-Wl,-rpath," + libdir,
                "-ltorch", "-ltorch_cpu", "-lc10", "-lc10_hip", "-ltorch_hip"]
        _run(link)
        # a launcher declared in kernels.h but defined inside an anonymous namespace (or
        # not at all) links fine into a shared object and only fails at dlopen on the GPU
        # box: refuse the build here instead
        und = subprocess.run(["nm", "-D", "--undefined-only", "-C", so + ".tmp"], capture_output=True, text=True)
        missing = [ln.split(None, 1)[-1] for ln in und.stdout.splitlines() if "hipserve::" in ln]
        if missing:
            os.remove(so + ".tmp")
            raise RuntimeError("hipserve/_C.so has undefined hipserve symbols: " + "; ".join(missing))
        os.replace(so + ".tmp", so)
    return so


def build_runtime(force: bool = False, verbose: bool = False) -> str:
    """Build hipserve/_runtime.so: native CPU runtime (block allocator, batch
    builder, shared-memory rings) via the CPython C API / pybind11."""
    srcs = sorted(glob.glob(os.path.join(CSRC, "runtime", "*.cpp")))
    if not srcs:
        return ""
    import pybind11

    os.makedirs(BUILD, exist_ok=True)
    so = os.path.join(PKG, "_runtime" + (sysconfig.get_config_var("EXT_SUFFIX") or ".so"))
    flags = ["-O3", "-std=c++17", "-fPIC", "-shared", "-Wall", "-Wno-sign-compare",
             "-I", pybind11.get_include(), "-I", sysconfig.get_paths()["include"],
             "-I", os.path.join(CSRC, "include")]
    deps = srcs + sorted(glob.glob(os.path.join(CSRC, "runtime", "*.h")))
    want = _stamp(deps, flags)
    stamp = os.path.join(BUILD, "runtime.stamp")
    if not force and os.path.exists(so) and os.path.exists(stamp) and open(stamp).read() == want:
        return so
    _run(["g++", *flags, *srcs, "-o", so + ".tmp", "-lpthread", "-lrt"])
    os.replace(so + ".tmp", so)
    with open(stamp, "w") as f:
        f.write(want)
    if verbose:
        print(f"[hipserve build] {os.path.relpath(so, ROOT)}", flush=True)
    return so


SANITIZERS = {
    # ThreadSanitizer: the shm ring's acquire/release protocol between threads
    "thread": ["-fsanitize=thread"],
    # AddressSanitizer + UBSan: out-of-bounds slot copies, pool bookkeeping
    "address": ["-fsanitize=address,undefined", "-fno-omit-frame-pointer", "-fno-sanitize-recover=all"],
}


def build_sanitizer_test(kind: str, verbose: bool = False) -> str:
    """Host-only build of csrc/tests/runtime_stress.cpp (native runtime cores, no
    Python, no GPU) under a sanitizer; returns the binary path. GPU-side
    sanitizers are not available on the MI355X pool (no xnack+), so the
    sanitizers cover the host runtime; kernels are checked by the numerics tests."""
    if kind not in SANITIZERS:
        raise ValueError(f"sanitizer {kind!r}: one of {sorted(SANITIZERS)}")
    out_dir = os.path.join(ROOT, "build", "san")
    os.makedirs(out_dir, exist_ok=True)
    src = os.path.join(CSRC, "tests", "runtime_stress.cpp")
    deps = [src] + sorted(glob.glob(os.path.join(CSRC, "runtime", "*.h")))
    flags = ["-O1", "-g", "-std=c++17", *SANITIZERS[kind], "-pthread"]
    exe = os.path.join(out_dir, f"runtime_stress_{kind}")
    want = _stamp(deps, flags)
    stamp = exe + ".stamp"
    if os.path.exists(exe) and os.path.exists(stamp) and open(stamp).read() == want:
        return exe
    _run(["g++", *flags, src, "-o", exe, "-lrt"])
    with open(stamp, "w") as f:
        f.write(want)
    if verbose:
        print(f"[hipserve build] {os.path.relpath(exe, ROOT)}", flush=True)
    return exe


def build_all(force: bool = False, jobs: int | None = None, verbose: bool = True):
    jobs = jobs or int(os.environ.get("MAX_JOBS", "8"))
    rt = build_runtime(force=force, verbose=verbose)
    so = build_kernels(force=force, jobs=jobs, verbose=verbose)
    return so, rt


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--force", action="store_true")
    ap.add_argument("-j", "--jobs", type=int, default=None)
    ap.add_argument("--sanitize", action="append", choices=sorted(SANITIZERS),
                    help="also build the native-runtime stress test under this sanitizer")
    a = ap.parse_args(argv)
    for kind in a.sanitize or []:
        print(build_sanitizer_test(kind, verbose=True))
    so, rt = build_all(force=a.force, jobs=a.jobs)
    print(so)
    if rt:
        print(rt)


if __name__ == "__main__":
    sys.exit(main())
