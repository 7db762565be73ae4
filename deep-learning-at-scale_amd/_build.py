"""In-tree build of the native libraries (gfx950 only).

``build()`` compiles

* ``csrc/*.hip``  with ``hipcc --offload-arch=gfx950`` (pure HIP, no torch headers),
* ``csrc/binding.cpp`` with ``g++`` against the installed PyTorch-ROCm headers,

and links them into ``wellflow/_C.so`` (a pybind11 module).  It also builds the native
runtime library ``wellflow/_runtime.so`` (C++ CSV reader / window batcher / prefetcher,
``csrc/runtime/*.cpp``, ctypes ABI) when its sources exist.

Builds are incremental (mtime-based) and parallel; the artefacts live inside the package
so they travel with the repository snapshot to the GPU box (a JIT cache under ~/.cache
would not).  There is no hipify step, no CUDA path and no fallback: on a GPU box the ops
import ``_C`` and fail loudly if it is missing.
"""
from __future__ import annotations

import concurrent.futures as cf
import glob
import os
import subprocess
import sys
import sysconfig

PKG_DIR = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(PKG_DIR, "csrc")
BUILD_DIR = os.path.join(PKG_DIR, "build")
EXT_PATH = os.path.join(PKG_DIR, "_C.so")
RUNTIME_PATH = os.path.join(PKG_DIR, "_runtime.so")
ROCM = os.environ.get("ROCM_PATH", "/opt/rocm")
ARCH = "gfx950"

HIPCC_FLAGS = [
    f"--offload-arch={ARCH}",
    "-O3",
    "-std=c++17",
    "-fPIC",
    "-munsafe-fp-atomics",  # float atomicAdd -> global_atomic_add_f32 (no CAS loop)
    "-Wno-unused-result",
]


def _torch_flags():
    import torch
    from torch.utils import cpp_extension as ce

    inc = ce.include_paths("cuda")
    flags = [f"-I{p}" for p in inc]
    flags += [
        "-D__HIP_PLATFORM_AMD__=1",
        "-DUSE_ROCM=1",
        "-DTORCH_EXTENSION_NAME=_C",
        "-DTORCH_API_INCLUDE_EXTENSION_H",
        f"-D_GLIBCXX_USE_CXX11_ABI={int(torch.compiled_with_cxx11_abi())}",
        f"-I{sysconfig.get_paths()['include']}",
    ]
    libdir = os.path.join(os.path.dirname(torch.__file__), "lib")
    ldflags = [
        f"-L{libdir}",
        "-lc10",
        "-ltorch",
        "-ltorch_cpu",
        "-ltorch_python",
        "-lc10_hip",
        "-ltorch_hip",
        "-lamdhip64",  # torch's bundled HIP runtime (same soname as /opt/rocm's)
        f"-Wl,-rpath,{libdir}",
    ]
    return flags, ldflags


def _stale(target: str, deps) -> bool:
    if not os.path.exists(target):
        return True
    t = os.path.getmtime(target)
    return any(os.path.getmtime(d) > t for d in deps)


def _local_deps(src: str, seen=None) -> list:
    """The quoted #include files of ``src`` (transitively, csrc-local only): a header edit
    rebuilds only the sources that include it (the persistent LSTM kernels alone take
    minutes to compile)."""
    import re

    seen = set() if seen is None else seen
    d = os.path.dirname(src)
    with open(src) as f:
        for inc in re.findall(r'^\s*#\s*include\s+"([^"]+)"', f.read(), re.M):
            p = os.path.normpath(os.path.join(d, inc))
            if os.path.exists(p) and p not in seen:
                seen.add(p)
                _local_deps(p, seen)
    return sorted(seen)


def _variants(src: str) -> list:
    """[(object tag, -D flags)]: one object per variant listed in the source's
    ``// wf-build-variants: -DA=1 -DB=2 | -DA=3 ...`` lines (instantiation sources compile in
    parallel, one slow template instantiation each), else one plain object."""
    out = []
    with open(src) as f:
        for line in f:
            if line.startswith("// wf-build-variants:"):
                for v in line.split(":", 1)[1].split("|"):
                    defs = v.split()
                    tag = "." + "_".join(d[2:].replace("=", "") for d in defs)
                    out.append((tag, defs))
    return out or [("", [])]


def _run(cmd, verbose):
    if verbose:
        print(" ".join(cmd), flush=True)
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"build failed: {' '.join(cmd)}\n{r.stdout}\n{r.stderr}")
    return r


def build(verbose: bool = False, jobs: int | None = None) -> str:
    """Compile every HIP source for gfx950 and link ``_C.so``; returns its path."""
    os.makedirs(BUILD_DIR, exist_ok=True)
    hip_srcs = sorted(glob.glob(os.path.join(CSRC, "*.hip")))
    tflags, ldflags = _torch_flags()
    hipcc = os.path.join(ROCM, "bin", "hipcc")
    jobs = jobs or min(8, os.cpu_count() or 4)

    tasks = []
    objs = []
    # WELLFLOW_DIAG_BUILD=1: also the timing-only diagnostic kernel variants (WELLFLOW_PF_DBG,
    # tools/pf_time.py, pb_time.py, *_timeline.py); separate objects, so switching is a relink
    # (=N or =N,M,..: only those WELLFLOW_PF_DBG variants, for a quick diagnostic build)
    dval = os.environ.get("WELLFLOW_DIAG_BUILD", "0")
    diag = dval not in ("", "0")
    for src in hip_srcs:
        deps = [src] + _local_deps(src)
        for tag, defs in _variants(src):
            vals = [int(v) for v in dval.split(",")] if diag else []
            defs = defs + (["-DWF_DIAG"] + ([f"-DWF_DIAG_SET={','.join(map(str, vals))}"] if dval != "1" else [])
                           if diag else [])
            dtag = (".diag" if dval == "1" else ".diag" + "_".join(map(str, vals))) if diag else ""
            obj = os.path.join(BUILD_DIR, os.path.basename(src) + tag + dtag + ".o")
            objs.append(obj)
            if _stale(obj, deps):
                tasks.append([hipcc, *HIPCC_FLAGS, *defs, f"-I{CSRC}", "-c", src, "-o", obj])
    bsrc = os.path.join(CSRC, "binding.cpp")
    bobj = os.path.join(BUILD_DIR, "binding.cpp.o")
    objs.append(bobj)
    if _stale(bobj, [bsrc] + _local_deps(bsrc)):
        tasks.append(["g++", "-O2", "-std=c++17", "-fPIC", f"-I{CSRC}", *tflags, "-c", bsrc, "-o", bobj])

    with cf.ThreadPoolExecutor(max_workers=jobs) as ex:
        for f in [ex.submit(_run, t, verbose) for t in tasks]:
            f.result()

    # the link is stale when an object is newer than _C.so OR the object SET changed (a switch
    # between the production and a WF_DIAG build whose objects all exist already relinks too:
    # the stamp next to _C.so names the objects it was linked from; round-3 ADVICE)
    stamp = EXT_PATH + ".objs"
    want = "\n".join(os.path.basename(o) for o in objs) + "\n"
    have = open(stamp).read() if os.path.exists(stamp) else ""
    if _stale(EXT_PATH, objs) or have != want:
        tmp = EXT_PATH + ".tmp"
        _run(["g++", "-shared", "-o", tmp, *objs, *ldflags], verbose)
        os.replace(tmp, EXT_PATH)
        with open(stamp, "w") as f:
            f.write(want)
    build_runtime(verbose)
    return EXT_PATH


def build_runtime(verbose: bool = False) -> str | None:
    """Native host runtime (C++17, no GPU code): CSV parsing, windowing, prefetch."""
    srcs = sorted(glob.glob(os.path.join(CSRC, "runtime", "*.cpp")))
    if not srcs:
        return None
    hdrs = glob.glob(os.path.join(CSRC, "runtime", "*.h"))
    if _stale(RUNTIME_PATH, srcs + hdrs):
        tmp = RUNTIME_PATH + ".tmp"
        _run(["g++", "-O3", "-std=c++17", "-fPIC", "-shared", "-pthread", *srcs, "-o", tmp], verbose)
        os.replace(tmp, RUNTIME_PATH)
    return RUNTIME_PATH


if __name__ == "__main__":
    print(build(verbose="-v" in sys.argv))
