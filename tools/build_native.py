#!/usr/bin/env python3
"""Build the package's single native extension (``apex._C``) for gfx950.

Why not ``torch.utils.cpp_extension.CUDAExtension``: on ROCm it runs hipify over the sources;
ours are HIP/CDNA4-native already, so we drive ``hipcc`` directly:

* ``csrc/**/*.hip``  -> device translation units, torch-free (fast to compile), ``--offload-arch=gfx950``
* ``csrc/bindings/*.cpp`` -> pybind/torch host code
* link -> ``rocm-apex_amd/_C.<abi>.so`` IN-TREE (it travels to the GPU box with the repo snapshot)

Incremental: an object is rebuilt when its source or any header under csrc/ is newer.

Per-extension selection (the reference's ``setup.py --cpp_ext --cuda_ext --fast_layer_norm ...``
flags, /root/reference/setup.py:87-555): ``--extensions norm,gemm`` or
``APEX_AMD_EXTENSIONS=norm,gemm`` builds the always-on core (multi-tensor engine, amp_C) plus
the named subsystems only; the Python side sees the others as absent (``apex._native.submodule``
returns None and the op raises on a GPU tensor).  Names: see ``EXTENSIONS``.

Usage: ``python tools/build_native.py [-j N] [--clean] [--verbose] [--extensions a,b] [--out PATH]``
"""
from __future__ import annotations

import argparse
import concurrent.futures as cf
import os
import shutil
import subprocess
import sys
import sysconfig
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "rocm-apex_amd")
CSRC = os.path.join(PKG, "csrc")
BUILD = os.path.join(ROOT, "build", "native")
ARCH = os.environ.get("APEX_AMD_ARCH", "gfx950")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")

# optional subsystems: name -> (binding file, device source dirs under csrc/)
EXTENSIONS = {
    "norm": ("norm.cpp", ("norm",)),
    "softmax": ("softmax.cpp", ("softmax",)),
    "syncbn": ("syncbn.cpp", ("syncbn",)),
    "gemm": ("gemm.cpp", ("gemm",)),  # + lt_epilogue.cpp (hipBLASLt epilogue GEMMs)
    "xentropy": ("xentropy.cpp", ("xentropy",)),
    "attn": ("attn.cpp", ("attn",)),
    "bn_nhwc": ("bn_nhwc.cpp", ("groupbn",)),
    "conv": ("conv.cpp", ("conv",)),
    "contrib": ("contrib.cpp", ("comm", "pool", "transducer", "transformer")),
}
CORE_DIRS = ("mta",)

# binding file -> macro that module.cpp keys on
SUBSYSTEMS = {
    "norm.cpp": "APEX_AMD_WITH_NORM",
    "softmax.cpp": "APEX_AMD_WITH_SOFTMAX",
    "syncbn.cpp": "APEX_AMD_WITH_SYNCBN",
    "gemm.cpp": "APEX_AMD_WITH_GEMM",
    "xentropy.cpp": "APEX_AMD_WITH_XENTROPY",
    "attn.cpp": "APEX_AMD_WITH_ATTN",
    "contrib.cpp": "APEX_AMD_WITH_CONTRIB",
    "bn_nhwc.cpp": "APEX_AMD_WITH_BN_NHWC",
    "conv.cpp": "APEX_AMD_WITH_CONV",
}


def ext_suffix() -> str:
    return sysconfig.get_config_var("EXT_SUFFIX") or ".so"


def output_path(out=None) -> str:
    return out or os.environ.get("APEX_AMD_OUT") or os.path.join(PKG, "_C" + ext_suffix())


def torch_paths():
    import torch  # noqa: WPS433 (build-time dependency)

    tdir = os.path.dirname(torch.__file__)
    inc = [os.path.join(tdir, "include"), os.path.join(tdir, "include", "torch", "csrc", "api", "include")]
    abi = int(torch._C._GLIBCXX_USE_CXX11_ABI)
    return tdir, inc, abi


def selected_extensions(spec=None):
    spec = spec if spec is not None else os.environ.get("APEX_AMD_EXTENSIONS", "all")
    if spec in ("", "all"):
        return sorted(EXTENSIONS)
    names = sorted({n.strip() for n in spec.split(",") if n.strip()})
    bad = [n for n in names if n not in EXTENSIONS]
    if bad:
        raise RuntimeError(f"unknown extension(s) {bad}; choose from {sorted(EXTENSIONS)}")
    return names


def sources(extensions=None):
    names = selected_extensions(extensions)
    dirs = set(CORE_DIRS) | {d for n in names for d in EXTENSIONS[n][1]}
    skip_bind = {EXTENSIONS[n][0] for n in EXTENSIONS if n not in names}
    hip, cpp = [], []
    for d, _, files in os.walk(CSRC):
        top = os.path.relpath(d, CSRC).split(os.sep)[0]
        for f in sorted(files):
            p = os.path.join(d, f)
            if f.endswith(".hip") and top in dirs:
                hip.append(p)
            elif f.endswith(".cpp") and top == "bindings" and f not in skip_bind:
                cpp.append(p)
    return sorted(hip), sorted(cpp)


def newest_header() -> float:
    t = 0.0
    for d, _, files in os.walk(CSRC):
        for f in files:
            if f.endswith((".h", ".hpp", ".cuh", ".inc")):
                t = max(t, os.path.getmtime(os.path.join(d, f)))
    return t


_INCLUDE_RX = None


def header_deps(path: str, seen=None) -> set:
    """Transitive set of this package's headers a source includes (``#include "apex_amd/..."``
    or a relative quote include), so a header edit rebuilds only the units that use it."""
    global _INCLUDE_RX
    import re

    if _INCLUDE_RX is None:
        _INCLUDE_RX = re.compile(r'^\s*#\s*include\s*"([^"]+)"', re.M)
    seen = set() if seen is None else seen
    try:
        text = open(path, encoding="utf-8", errors="replace").read()
    except OSError:
        return seen
    for inc in _INCLUDE_RX.findall(text):
        for base in (os.path.join(CSRC, "include"), os.path.dirname(path)):
            cand = os.path.normpath(os.path.join(base, inc))
            if os.path.isfile(cand):
                if cand not in seen:
                    seen.add(cand)
                    header_deps(cand, seen)
                break
    return seen


def newest_dep(src: str) -> float:
    return max([os.path.getmtime(src)] + [os.path.getmtime(h) for h in header_deps(src)])


def obj_for(src: str, build_dir: str = BUILD) -> str:
    rel = os.path.relpath(src, CSRC).replace(os.sep, "__")
    return os.path.join(build_dir, rel + ".o")


def compile_cmds(verbose: bool, extensions=None, out=None, build_dir=BUILD, defines=()):
    tdir, tinc, abi = torch_paths()
    py_inc = sysconfig.get_paths()["include"]
    hip, cpp = sources(extensions)
    present = {os.path.basename(p) for p in cpp}
    macros = [f"-D{m}" for f, m in SUBSYSTEMS.items() if f in present]
    common = ["-std=c++17", "-O3", "-fPIC", f"-I{os.path.join(CSRC, 'include')}", "-Wno-unused-result",
              "-Wno-deprecated-declarations", "-Wno-unused-command-line-argument", *[f"-D{d}" for d in defines]]
    dev = [HIPCC, *common, f"--offload-arch={ARCH}", "-munsafe-fp-atomics", "-ffp-contract=fast",
           "--no-offload-compress", "-x", "hip"]
    host = [HIPCC, *common, "-D__HIP_PLATFORM_AMD__=1", "-DUSE_ROCM=1", "-DTORCH_EXTENSION_NAME=_C",
            "-DTORCH_API_INCLUDE_EXTENSION_H", f"-D_GLIBCXX_USE_CXX11_ABI={abi}", *macros,
            *[f"-isystem{p}" for p in tinc], f"-isystem{py_inc}", "-fvisibility=hidden"]
    jobs = []
    for s in hip:
        jobs.append((s, [*dev, "-c", s, "-o", obj_for(s, build_dir)]))
    for s in cpp:
        jobs.append((s, [*host, "-c", s, "-o", obj_for(s, build_dir)]))
    link = [HIPCC, "-shared", "-fPIC", f"--offload-arch={ARCH}", "-o", output_path(out),
            *[obj_for(s, build_dir) for s, _ in jobs],
            f"-L{os.path.join(tdir, 'lib')}", "-lc10", "-lc10_hip", "-ltorch", "-ltorch_cpu", "-ltorch_hip",
            "-ltorch_python", "-lamdhip64", "-L/opt/rocm/lib", "-lhipblaslt", "-Wl,-rpath,/opt/rocm/lib",
            f"-Wl,-rpath,{os.path.join(tdir, 'lib')}"]
    return jobs, link


def run(cmd, verbose):
    if verbose:
        print(" ".join(cmd), flush=True)
    t0 = time.time()
    r = subprocess.run(cmd, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True)
    return r.returncode, r.stdout, time.time() - t0


def build(jobs_n: int | None = None, clean: bool = False, verbose: bool = False, extensions=None,
          out=None, defines=()) -> str:
    names = selected_extensions(extensions)
    # a partial selection / extra defines get their own object dir so they never poison the
    # full build's objects
    build_dir = BUILD if names == sorted(EXTENSIONS) else os.path.join(BUILD, "sel_" + "_".join(names))
    if defines:
        build_dir = os.path.join(build_dir, "def_" + "_".join(d.replace("=", "-") for d in sorted(defines)))
    if clean and os.path.isdir(build_dir):
        shutil.rmtree(build_dir)
    os.makedirs(build_dir, exist_ok=True)
    jobs, link = compile_cmds(verbose, extensions, out, build_dir, tuple(defines))
    # module.cpp's registrations depend on which subsystem bindings exist (-D macros): rebuild it
    # whenever that set changes
    _, cpp = sources(extensions)
    present = sorted(os.path.basename(p) for p in cpp)
    stamp = os.path.join(build_dir, "subsystems.stamp")
    prev = open(stamp).read() if os.path.exists(stamp) else ""
    subsystems_changed = prev != ",".join(present)
    todo = []
    for src, cmd in jobs:
        o = obj_for(src, build_dir)
        stale = not os.path.exists(o) or os.path.getmtime(o) < newest_dep(src)
        if stale or (subsystems_changed and src.endswith("module.cpp")):
            todo.append((src, cmd))
    n = jobs_n or min(len(todo) or 1, max(1, (os.cpu_count() or 4)))
    failed = []
    if todo:
        print(f"[build_native] compiling {len(todo)} translation unit(s) for {ARCH} with {n} job(s)", flush=True)
        with cf.ThreadPoolExecutor(max_workers=n) as ex:
            futs = {ex.submit(run, cmd, verbose): src for src, cmd in todo}
            for f in cf.as_completed(futs):
                rc, log, dt = f.result()
                src = os.path.relpath(futs[f], ROOT)
                if rc != 0:
                    failed.append(src)
                    print(f"[build_native] FAILED {src}\n{log}", flush=True)
                else:
                    print(f"[build_native] {src} ({dt:.1f}s)", flush=True)
                    if log.strip() and verbose:
                        print(log)
    if failed:
        raise RuntimeError(f"native build failed: {failed}")
    with open(stamp, "w") as f:
        f.write(",".join(present))
    out = output_path(out)
    objs_newest = max(os.path.getmtime(obj_for(s, build_dir)) for s, _ in jobs)
    if todo or not os.path.exists(out) or os.path.getmtime(out) < objs_newest:
        rc, log, dt = run(link, verbose)
        if rc != 0:
            print(log)
            raise RuntimeError("native link failed")
        print(f"[build_native] linked {os.path.relpath(out, ROOT)} ({dt:.1f}s)", flush=True)
    return out


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("-j", type=int, default=None)
    ap.add_argument("--clean", action="store_true")
    ap.add_argument("--verbose", "-v", action="store_true")
    ap.add_argument("--extensions", default=None, help="comma list of " + ",".join(sorted(EXTENSIONS)))
    ap.add_argument("--out", default=None, help="output .so path (default: in-tree)")
    ap.add_argument("--define", "-D", action="append", default=[],
                    help="extra preprocessor define for an A/B variant build (use with --out)")
    a = ap.parse_args(argv)
    if a.define and not a.out:
        ap.error("--define builds a variant: give it its own --out path")
    try:
        build(a.j, a.clean, a.verbose, a.extensions, a.out, a.define)
    except RuntimeError as e:
        print(f"[build_native] {e}", file=sys.stderr)
        return 1
    return 0


if __name__ == "__main__":
    sys.exit(main())
