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

Build integrity is content-based, not mtime-based: every module carries a
stamp ``HETSEQ_SRC_HASH=<sha256>`` (a data symbol linked into the ``.so``)
over its sources, shared headers, compiler flags and target arch.  A module is
rebuilt exactly when its embedded stamp differs from the hash of the tree it
sits in, and ``hetseq_amd/ops/_C.py`` refuses to import a module whose stamp
does not match (it rebuilds first, or raises with HETSEQ_NO_AUTOBUILD=1), so a
loaded ``_hip.so`` is always the code of the sources next to it.  Objects are
cached per translation unit under ``build/native`` with the same content hash.
``python -m hetseq_amd.csrc.build`` builds everything.
"""
from __future__ import annotations

import concurrent.futures as cf
import hashlib
import os
import re
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


def _digest(paths, flags, extra=""):
    """sha256 over the contents of ``paths`` (sorted by name), the compiler flags and ``extra``."""
    h = hashlib.sha256()
    h.update(extra.encode())
    for f in flags:
        h.update(b"\0F" + f.encode())
    for p in sorted(paths, key=os.path.basename):
        h.update(b"\0P" + os.path.basename(p).encode() + b"\0")
        with open(p, "rb") as fh:
            h.update(fh.read())
    return h.hexdigest()


_STAMP_RE = re.compile(rb"HETSEQ_SRC_HASH=([0-9a-f]{64})")


def embedded_hash(so_path):
    """The source stamp linked into a built module (None: missing file or no stamp)."""
    try:
        with open(so_path, "rb") as fh:
            m = _STAMP_RE.search(fh.read())
    except OSError:
        return None
    return m.group(1).decode() if m else None


def _run(cmd, verbose):
    if verbose:
        print(" ".join(cmd), flush=True)
    r = subprocess.run(cmd, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True)
    if r.returncode != 0:
        raise RuntimeError("native build failed:\n" + " ".join(cmd) + "\n" + r.stdout)
    return r.stdout


def _headers(dirpath):
    return [os.path.join(dirpath, f) for f in os.listdir(dirpath) if f.endswith((".h", ".hpp", ".cuh"))]


# per-translation-unit extra flags (kept in the object and module hashes)
SOURCE_FLAGS: dict = {}


_INC_RE = re.compile(r'^\s*#\s*include\s*"([^"]+)"', re.M)


def _included(src, headers):
    """The module headers ``src`` includes, directly or through another of them (quoted includes):
    an object is rebuilt when one of THOSE changes, not when any header of the directory does."""
    by_name = {os.path.basename(h): h for h in headers}
    seen, todo = [], [src]
    while todo:
        with open(todo.pop()) as fh:
            text = fh.read()
        for inc in _INC_RE.findall(text):
            h = by_name.get(os.path.basename(inc))
            if h is not None and h not in seen:
                seen.append(h)
                todo.append(h)
    return seen


def _compile_objs(compiler, flags, sources, headers, objdir, verbose, jobs):
    """Compile each source whose content hash (source + headers + flags) differs from the one
    recorded next to its object file."""
    os.makedirs(objdir, exist_ok=True)
    todo, objs = [], []
    for src in sources:
        obj = os.path.join(objdir, os.path.basename(src) + ".o")
        objs.append(obj)
        want = _digest([src] + _included(src, headers), [compiler] + flags + SOURCE_FLAGS.get(os.path.basename(src), []))
        try:
            with open(obj + ".hash") as fh:
                have = fh.read().strip()
        except OSError:
            have = None
        if have != want or not os.path.exists(obj):
            todo.append((src, obj, want))
    if todo:
        with cf.ThreadPoolExecutor(max_workers=max(1, jobs)) as ex:
            futs = [ex.submit(_run, [compiler] + flags + SOURCE_FLAGS.get(os.path.basename(s), []) + ["-c", s, "-o", o],
                              verbose) for s, o, _ in todo]
            for f in futs:
                f.result()
        for _, o, want in todo:
            with open(o + ".hash", "w") as fh:
                fh.write(want)
    return objs


def _stamp_obj(name, digest, objdir, verbose):
    """Object file defining the module's source stamp (a plain data symbol, kept by the linker)."""
    os.makedirs(objdir, exist_ok=True)
    src = os.path.join(objdir, "stamp_%s.cpp" % name)
    with open(src, "w") as fh:
        fh.write('extern "C" __attribute__((visibility("default"), used)) const char hetseq_src_stamp_%s[] = '
                 '"HETSEQ_SRC_HASH=%s";\n' % (name.strip("_"), digest))
    obj = src[:-4] + ".o"
    _run(["g++", "-fPIC", "-c", src, "-o", obj], verbose)
    return obj


def _link(compiler, objs, out, ldflags, verbose):
    tmp = "%s.tmp.%d" % (out, os.getpid())  # per-process: two builders never share a half-written file
    try:
        _run([compiler, "-shared", "-o", tmp] + objs + ldflags, verbose)
        os.replace(tmp, out)  # atomic: a running process never sees a half-written .so
    finally:
        if os.path.exists(tmp):
            os.unlink(tmp)


class _BuildLock(object):
    """Inter-process lock around one module's build (``fcntl.flock`` on a file in BUILD_DIR).

    Every rank of a multi-process launch may find the same stale stamp at import; without the lock
    they would compile into the same object directory and link over each other.  The holder builds;
    the others wait, then find the fresh stamp and return without building."""

    def __init__(self, name):
        os.makedirs(BUILD_DIR, exist_ok=True)
        self.path = os.path.join(BUILD_DIR, ".lock" + name)
        self.fh = None

    def __enter__(self):
        import fcntl

        self.fh = open(self.path, "a+")
        fcntl.flock(self.fh.fileno(), fcntl.LOCK_EX)
        return self

    def __exit__(self, *exc):
        import fcntl

        fcntl.flock(self.fh.fileno(), fcntl.LOCK_UN)
        self.fh.close()
        return False


def _build_module(name, compiler, flags, sources, headers, ldflags, objdir, verbose, jobs, out=None,
                  link_compiler=None):
    """Build ``hetseq_amd/<name>.so`` unless its embedded stamp already matches the tree."""
    out = out or os.path.join(PKG, name + EXT)
    digest = module_hash(name)
    if embedded_hash(out) == digest:
        return out
    with _BuildLock(name):
        if embedded_hash(out) == digest:  # another process built it while this one waited
            return out
        objs = _compile_objs(compiler, flags, sources, headers, objdir, verbose, jobs)
        objs.append(_stamp_obj(name, digest, objdir, verbose))
        _link(link_compiler or compiler, objs, out, ldflags, verbose)
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
    objs = _compile_objs(SAN_CXX, base + pyinc, [nsrc], [], os.path.join(outdir, "obj-native"), verbose, jobs)
    outs = [os.path.join(outdir, "_native" + EXT)]
    _link(SAN_CXX, objs, outs[0], ["-pthread"] + SAN_FLAGS, verbose)
    inc, lib = os.path.join(HDF5_ROOT, "include"), os.path.join(HDF5_ROOT, "lib")
    if os.path.exists(os.path.join(inc, "hdf5.h")):
        hsrc = os.path.join(HERE, "native", "h5shard.cpp")
        objs = _compile_objs(SAN_CXX, base + ["-I" + inc] + pyinc, [hsrc], [],
                                      os.path.join(outdir, "obj-h5"), verbose, jobs)
        outs.append(os.path.join(outdir, "_h5" + EXT))
        # libhdf5 by path, not -L (the HDF5 prefix ships older sanitizer runtimes and libstdc++);
        # the system libstdc++ directory is searched before the HDF5 prefix at run time
        sysdir = "/usr/lib/x86_64-linux-gnu"
        _link(SAN_CXX, objs, outs[1], ["-pthread"] + SAN_FLAGS + [os.path.join(lib, "libhdf5.so"),
              "-Wl,-rpath," + sysdir + ":" + lib], verbose)
    return outs


def hip_sources():
    kdir = os.path.join(HERE, "kernels")
    return sorted(os.path.join(kdir, f) for f in os.listdir(kdir) if f.endswith((".hip", ".cpp")))


def _torch_lib():
    """torch's bundled ROCm runtime directory: the comm engine links the SAME librccl / libamdhip64
    that torch loaded (one RCCL instance per process)."""
    import importlib.util

    spec = importlib.util.find_spec("torch")
    return os.path.join(os.path.dirname(spec.origin), "lib")


def _spec(name):
    """(compiler, flags, sources, headers, ldflags, objdir) of one in-tree module."""
    pyinc = ["-I" + p for p in _py_includes()]
    host = ["-O3", "-std=c++17", "-fPIC", "-fvisibility=hidden", "-Wall"]
    if name == "_native":
        return ("g++", host + pyinc, [os.path.join(HERE, "native", "batcher.cpp")], [], ["-pthread"],
                os.path.join(BUILD_DIR, "native"))
    if name == "_h5":
        inc, lib = os.path.join(HDF5_ROOT, "include"), os.path.join(HDF5_ROOT, "lib")
        if not os.path.exists(os.path.join(inc, "hdf5.h")):
            raise RuntimeError("libhdf5 headers not found under %s (set HETSEQ_HDF5_ROOT)" % HDF5_ROOT)
        # Link the real soname file so the loader never needs the dev symlink.  static libstdc++:
        # the rpath to the HDF5 prefix would otherwise pick its older libstdc++
        return ("g++", host + ["-I" + inc] + pyinc, [os.path.join(HERE, "native", "h5shard.cpp")], [],
                ["-pthread", "-static-libstdc++", "-static-libgcc", "-L" + lib, "-lhdf5", "-Wl,-rpath," + lib],
                os.path.join(BUILD_DIR, "h5"))
    if name == "_hip":
        hipcc = shutil.which("hipcc") or os.path.join(ROCM, "bin", "hipcc")
        kdir = os.path.join(HERE, "kernels")
        flags = ["-O3", "-std=c++17", "-fPIC", "-fvisibility=hidden", "--offload-arch=" + ARCH, "-munsafe-fp-atomics",
                 "-Wno-unused-result", "-I" + kdir] + pyinc
        return (hipcc, flags, hip_sources(), _headers(kdir),
                ["--offload-arch=" + ARCH, "-L" + os.path.join(ROCM, "lib"), "-lamdhip64"],
                os.path.join(BUILD_DIR, "hip-" + ARCH))
    if name == "_comm":
        tlib = _torch_lib()
        rccl = os.path.join(tlib, "librccl.so")
        if not os.path.exists(rccl):
            rccl = os.path.join(ROCM, "lib", "librccl.so")
        hip = os.path.join(tlib, "libamdhip64.so")
        if not os.path.exists(hip):
            hip = os.path.join(ROCM, "lib", "libamdhip64.so")
        flags = ["-O2", "-std=c++17", "-fPIC", "-fvisibility=hidden", "-Wall", "-D__HIP_PLATFORM_AMD__",
                 "-I" + os.path.join(ROCM, "include")] + pyinc
        return ("g++", flags, [os.path.join(HERE, "comm", "comm.cpp")], [],
                ["-pthread", rccl, hip, "-Wl,-rpath," + os.path.dirname(rccl)], os.path.join(BUILD_DIR, "comm"))
    raise KeyError(name)


MODULES = ("_native", "_h5", "_hip", "_comm")


def module_hash(name):
    """Content hash the module's embedded stamp must equal: its sources, shared headers,
    compiler, flags (include paths and target arch among them) and link flags."""
    cc, flags, srcs, hdrs, ld, _ = _spec(name)
    # directories dropped (same toolchain, different install prefix or PATH entry -> same stamp)
    extra = [f for src in srcs for f in ["SRC:" + os.path.basename(src)] + SOURCE_FLAGS.get(os.path.basename(src), [])]
    norm = [re.sub(r"/[^\s:]*/", "", f) for f in [cc] + flags + ["LD"] + ld + extra]
    return _digest(srcs + hdrs, norm, extra=name)


def stamp_status(name, so_path=None):
    """(embedded stamp, expected hash) of an in-tree module; equal means the .so is current."""
    return embedded_hash(so_path or os.path.join(PKG, name + EXT)), module_hash(name)


def _build(name, verbose, jobs):
    cc, flags, srcs, hdrs, ld, objdir = _spec(name)
    return _build_module(name, cc, flags, srcs, hdrs, ld, objdir, verbose, jobs)


def build_native(verbose=False, jobs=4):
    return _build("_native", verbose, jobs)


def build_h5(verbose=False, jobs=4):
    return _build("_h5", verbose, jobs)


def build_hip(verbose=False, jobs=8):
    return _build("_hip", verbose, jobs)


def build_comm(verbose=False, jobs=4):
    """``hetseq_amd/_comm*.so`` -- the RCCL gradient-communication engine (host C++, g++)."""
    return _build("_comm", verbose, jobs)


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
