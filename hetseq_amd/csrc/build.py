"""In-tree native build for hetseq_amd (no setuptools, no hipify, no JIT cache).

Four extension modules are produced next to the package sources so that
they travel with the repository snapshot to the GPU box:

* ``hetseq_amd/_native*.so`` -- host runtime (batcher), plain g++.
* ``hetseq_amd/_h5*.so``     -- HDF5 shard reader/writer/prefetcher, g++ + libhdf5.
* ``hetseq_amd/_hip*.so``    -- CDNA4 kernels, ``hipcc --offload-arch=gfx950``.
* ``hetseq_amd/_comm*.so``   -- RCCL gradient-communication engine (comm stream, watchdog).

The HIP module does not include any torch header: kernels are launched
through a thin pybind11 layer that takes raw device addresses and a
``hipStream_t`` handle (the Python side passes ``tensor.data_ptr()`` and
``torch.cuda.current_stream().cuda_stream``).  That keeps compile times in
seconds and avoids the torch C++ ABI altogether.

Each translation unit is compiled to an object file only when its source
(or any shared header) is newer than the object; objects compile in a
process pool.  ``python -m hetseq_amd.csrc.build`` builds everything.
"""
from __future__ import annotations

import concurrent.futures as cf
import os
import shutil
import subprocess
import sys
import sysconfig

HERE = os.path.dirname(os.path.abspath(__file__))
PKG = os.path.dirname(HERE)
BUILD_DIR = os.path.join(PKG, "..", "build", "native")
EXT = sysconfig.get_config_var("EXT_SUFFIX") or ".so"
ARCH = os.environ.get("HETSEQ_OFFLOAD_ARCH", "gfx950")
HDF5_ROOT = os.environ.get("HETSEQ_HDF5_ROOT", "/opt/conda")
ROCM = os.environ.get("ROCM_PATH", "/opt/rocm")


def _py_includes():
    import pybind11

    return [sysconfig.get_paths()["include"], pybind11.get_include()]


def _newer(target, deps):
    if not os.path.exists(target):
        return True
    t = os.path.getmtime(target)
    return any(os.path.getmtime(d) > t for d in deps)


def _run(cmd, verbose):
    if verbose:
        print(" ".join(cmd), flush=True)
    r = subprocess.run(cmd, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True)
    if r.returncode != 0:
        raise RuntimeError("native build failed:\n" + " ".join(cmd) + "\n" + r.stdout)
    return r.stdout


def _headers(dirpath):
    return [os.path.join(dirpath, f) for f in os.listdir(dirpath) if f.endswith((".h", ".hpp", ".cuh"))]


def _compile_objs(compiler, flags, sources, headers, objdir, verbose, jobs):
    os.makedirs(objdir, exist_ok=True)
    todo, objs = [], []
    for src in sources:
        obj = os.path.join(objdir, os.path.basename(src) + ".o")
        objs.append(obj)
        if _newer(obj, [src] + headers):
            todo.append((src, obj))
    if todo:
        with cf.ThreadPoolExecutor(max_workers=max(1, jobs)) as ex:
            futs = [ex.submit(_run, [compiler] + flags + ["-c", s, "-o", o], verbose) for s, o in todo]
            for f in futs:
                f.result()
    return objs, bool(todo)


def _link(compiler, objs, out, ldflags, verbose, force):
    if force or _newer(out, objs):
        tmp = out + ".tmp"
        _run([compiler, "-shared", "-o", tmp] + objs + ldflags, verbose)
        os.replace(tmp, out)  # atomic: a running process never sees a half-written .so


def build_native(verbose=False, jobs=4):
    src = os.path.join(HERE, "native", "batcher.cpp")
    if not _newer(os.path.join(PKG, "_native" + EXT), [src]):
        return os.path.join(PKG, "_native" + EXT)
    flags = ["-O3", "-std=c++17", "-fPIC", "-fvisibility=hidden", "-Wall"] + ["-I" + p for p in _py_includes()]
    objs, changed = _compile_objs("g++", flags, [src], [], os.path.join(BUILD_DIR, "native"), verbose, jobs)
    out = os.path.join(PKG, "_native" + EXT)
    _link("g++", objs, out, ["-pthread"], verbose, changed)
    return out


def build_h5(verbose=False, jobs=4):
    inc = os.path.join(HDF5_ROOT, "include")
    lib = os.path.join(HDF5_ROOT, "lib")
    if not os.path.exists(os.path.join(inc, "hdf5.h")):
        raise RuntimeError("libhdf5 headers not found under %s (set HETSEQ_HDF5_ROOT)" % HDF5_ROOT)
    src = os.path.join(HERE, "native", "h5shard.cpp")
    if not _newer(os.path.join(PKG, "_h5" + EXT), [src]):
        return os.path.join(PKG, "_h5" + EXT)
    flags = ["-O3", "-std=c++17", "-fPIC", "-fvisibility=hidden", "-Wall", "-I" + inc] + [
        "-I" + p for p in _py_includes()
    ]
    objs, changed = _compile_objs("g++", flags, [src], [], os.path.join(BUILD_DIR, "h5"), verbose, jobs)
    out = os.path.join(PKG, "_h5" + EXT)
    # Link the real soname file so the loader never needs the dev symlink.
    # static libstdc++: the rpath to the HDF5 prefix would otherwise pick its older libstdc++
    _link("g++", objs, out, ["-pthread", "-static-libstdc++", "-static-libgcc", "-L" + lib, "-lhdf5", "-Wl,-rpath," + lib],
          verbose, changed)
    return out


SAN_FLAGS = ["-O1", "-g", "-fno-omit-frame-pointer", "-fsanitize=address,undefined", "-fno-sanitize-recover=undefined",
             "-shared-libsan"]
SAN_CXX = os.path.join(ROCM, "lib", "llvm", "bin", "clang++")


def asan_runtime():
    """Path of the clang ASan runtime the sanitized modules need preloaded."""
    import glob

    hits = sorted(glob.glob(os.path.join(ROCM, "lib", "llvm", "lib", "clang", "*", "lib", "linux",
                                         "libclang_rt.asan-x86_64.so")))
    return hits[-1] if hits else None


def build_sanitized(outdir=None, verbose=False, jobs=4):
    """ASan+UBSan builds of the host runtime (batcher, HDF5 IO) for the sanitizer test.

    Built with the ROCm LLVM clang (its runtime copes with this kernel's
    high-entropy mmap layout; the gcc 11 runtime does not).  The modules keep
    their import names (``_native``, ``_h5``) but land in ``outdir`` (default
    ``build/native/asan``) so they never shadow the in-tree ones;
    ``tools/asan_native.py`` loads them with ``LD_PRELOAD=asan_runtime()``.
    Host code only: GPU sanitizers are not used on this platform.
    """
    outdir = outdir or os.path.join(BUILD_DIR, "asan")
    os.makedirs(outdir, exist_ok=True)
    pyinc = ["-I" + p for p in _py_includes()]
    base = ["-std=c++17", "-fPIC", "-Wall"] + SAN_FLAGS
    nsrc = os.path.join(HERE, "native", "batcher.cpp")
    objs, changed = _compile_objs(SAN_CXX, base + pyinc, [nsrc], [], os.path.join(outdir, "obj-native"), verbose, jobs)
    outs = [os.path.join(outdir, "_native" + EXT)]
    _link(SAN_CXX, objs, outs[0], ["-pthread"] + SAN_FLAGS, verbose, changed)
    inc, lib = os.path.join(HDF5_ROOT, "include"), os.path.join(HDF5_ROOT, "lib")
    if os.path.exists(os.path.join(inc, "hdf5.h")):
        hsrc = os.path.join(HERE, "native", "h5shard.cpp")
        objs, changed = _compile_objs(SAN_CXX, base + ["-I" + inc] + pyinc, [hsrc], [],
                                      os.path.join(outdir, "obj-h5"), verbose, jobs)
        outs.append(os.path.join(outdir, "_h5" + EXT))
        # libhdf5 by path, not -L (the HDF5 prefix ships older sanitizer runtimes and libstdc++);
        # the system libstdc++ directory is searched before the HDF5 prefix at run time
        sysdir = "/usr/lib/x86_64-linux-gnu"
        _link(SAN_CXX, objs, outs[1], ["-pthread"] + SAN_FLAGS + [os.path.join(lib, "libhdf5.so"),
              "-Wl,-rpath," + sysdir + ":" + lib], verbose, changed)
    return outs


def hip_sources():
    kdir = os.path.join(HERE, "kernels")
    return sorted(os.path.join(kdir, f) for f in os.listdir(kdir) if f.endswith((".hip", ".cpp")))


def build_hip(verbose=False, jobs=8):
    hipcc = shutil.which("hipcc") or os.path.join(ROCM, "bin", "hipcc")
    kdir = os.path.join(HERE, "kernels")
    out = os.path.join(PKG, "_hip" + EXT)
    if not _newer(out, hip_sources() + _headers(kdir)):
        return out  # the shipped module is current (object files need not travel with the tree)
    flags = [
        "-O3",
        "-std=c++17",
        "-fPIC",
        "-fvisibility=hidden",
        "--offload-arch=" + ARCH,
        "-munsafe-fp-atomics",
        "-Wno-unused-result",
        "-I" + kdir,
    ] + ["-I" + p for p in _py_includes()]
    objs, changed = _compile_objs(
        hipcc, flags, hip_sources(), _headers(kdir), os.path.join(BUILD_DIR, "hip-" + ARCH), verbose, jobs
    )
    out = os.path.join(PKG, "_hip" + EXT)
    _link(hipcc, objs, out, ["--offload-arch=" + ARCH, "-L" + os.path.join(ROCM, "lib"), "-lamdhip64"], verbose, changed)
    return out


def _torch_lib():
    """torch's bundled ROCm runtime directory: the comm engine links the SAME librccl / libamdhip64
    that torch loaded (one RCCL instance per process)."""
    import importlib.util

    spec = importlib.util.find_spec("torch")
    return os.path.join(os.path.dirname(spec.origin), "lib")


def build_comm(verbose=False, jobs=4):
    """``hetseq_amd/_comm*.so`` -- the RCCL gradient-communication engine (host C++, g++)."""
    src = os.path.join(HERE, "comm", "comm.cpp")
    out = os.path.join(PKG, "_comm" + EXT)
    if not _newer(out, [src]):
        return out
    tlib = _torch_lib()
    rccl = os.path.join(tlib, "librccl.so")
    if not os.path.exists(rccl):
        rccl = os.path.join(ROCM, "lib", "librccl.so")
    hip = os.path.join(tlib, "libamdhip64.so")
    if not os.path.exists(hip):
        hip = os.path.join(ROCM, "lib", "libamdhip64.so")
    flags = ["-O2", "-std=c++17", "-fPIC", "-fvisibility=hidden", "-Wall", "-D__HIP_PLATFORM_AMD__",
             "-I" + os.path.join(ROCM, "include")] + ["-I" + p for p in _py_includes()]
    objs, changed = _compile_objs("g++", flags, [src], [], os.path.join(BUILD_DIR, "comm"), verbose, jobs)
    _link("g++", objs, out, ["-pthread", rccl, hip, "-Wl,-rpath," + os.path.dirname(rccl)], verbose, changed)
    return out


def build_all(verbose=False, hip=True, h5=True):
    outs = [build_native(verbose)]
    if h5:
        outs.append(build_h5(verbose))
    if hip:
        outs.append(build_hip(verbose))
        outs.append(build_comm(verbose))
    return outs


if __name__ == "__main__":
    v = "-v" in sys.argv
    for o in build_all(verbose=v, hip="--no-hip" not in sys.argv):
        print("built", os.path.relpath(o, os.path.join(PKG, "..")))
