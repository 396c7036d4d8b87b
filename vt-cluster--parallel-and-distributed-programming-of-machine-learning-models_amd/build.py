"""In-tree native build: every HIP/C++ source under ``csrc/`` -> ``_C.so``.

No torch cpp_extension (it would run hipify over the sources), no CMake:
we drive ``hipcc --offload-arch=gfx950`` directly, one object per source,
compiled in parallel and cached by content hash, then link one shared
object against libtorch (whose bundled ``libamdhip64.so.7`` is the HIP
runtime the process already has loaded).

Usage:  python -m mift.build [--force] [--verbose] [--jobs N]
"""
import argparse
import concurrent.futures as cf
import hashlib
import os
import re
import subprocess
import sys
import sysconfig

HERE = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(HERE, "csrc")
BUILD_DIR = os.path.join(os.path.dirname(HERE), "build", "mift")
OUT = os.path.join(HERE, "_C.so")
ARCH = os.environ.get("MIFT_ARCH", "gfx950")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")


def _torch_paths():
    import torch
    root = os.path.dirname(torch.__file__)
    inc = [os.path.join(root, "include"), os.path.join(root, "include", "torch", "csrc", "api", "include")]
    lib = os.path.join(root, "lib")
    abi = int(torch._C._GLIBCXX_USE_CXX11_ABI)
    return inc, lib, abi


def _sources():
    srcs = []
    for dp, _, fs in os.walk(CSRC):
        for f in sorted(fs):
            if f.endswith((".hip", ".cpp")):
                srcs.append(os.path.join(dp, f))
    return sorted(srcs)


_INCLUDE_RE = re.compile(rb'^[ \t]*#[ \t]*include[ \t]*"([^"]+)"', re.M)


def _deps_digest(src):
    """sha256 over the local files ``src`` includes (``#include "..."``, recursively, resolved against
    the including file's directory, then csrc/): an object is rebuilt only when something it compiles
    changed (the GEMM translation units share gemm_impl.h; the other kernels do not see it)."""
    h = hashlib.sha256()
    seen, todo = set(), [os.path.abspath(src)]
    while todo:
        path = todo.pop()
        with open(path, "rb") as fh:
            text = fh.read()
        if path != os.path.abspath(src):
            h.update(os.path.relpath(path, CSRC).encode())
            h.update(text)
        for inc in _INCLUDE_RE.findall(text):
            name = inc.decode()
            for base in (os.path.dirname(path), os.path.dirname(os.path.dirname(path)), CSRC):
                cand = os.path.abspath(os.path.join(base, name))
                if os.path.exists(cand):
                    if cand not in seen:
                        seen.add(cand)
                        todo.append(cand)
                    break
    return h.hexdigest()


def _common_flags():
    inc, _, abi = _torch_paths()
    py_inc = sysconfig.get_paths()["include"]
    flags = ["-O3", "-std=c++17", "-fPIC", f"--offload-arch={ARCH}",
             f"-D_GLIBCXX_USE_CXX11_ABI={abi}", "-DTORCH_EXTENSION_NAME=_C",
             "-DTORCH_API_INCLUDE_EXTENSION_H", "-DUSE_ROCM=1",
             "-Wno-unused-result", "-Wno-deprecated-declarations", "-Wno-unused-command-line-argument",
             f"-I{CSRC}", f"-I{py_inc}"]
    for i in inc:
        flags.append(f"-isystem{i}")
    if os.environ.get("MIFT_DEBUG"):
        flags.append("-DMIFT_DEBUG=1")
    return flags


_TILE10 = "Li256ELi256ELi2ELi2E"  # gemm_nt_kernel<T, 256, 256, 2, 2, ...>: the 4-wave mainloop4 tile


def check_pinned_accumulators(remarks):
    """The 4-wave 256x256 tile keeps its 256 fp32 accumulators in AGPRs through inline-asm MFMAs
    (`"+a"` operands, gemm_impl.h mfma_acc).  Under register pressure the allocator may keep them in
    VGPRs instead and copy them into AGPRs around every asm statement: bit-identical output, but the
    OPT-2.7B step went 79 -> 514 ms when one extra live value in the epilogue did that (round 6).
    Returns the offending kernels' (name, AGPR count) from hipcc's kernel-resource-usage remarks."""
    bad, cur = [], None
    for line in remarks.splitlines():
        if "Function Name:" in line:
            cur = line.split("Function Name:", 1)[1].split()[0]
        elif cur and "gemm_nt_kernel" in cur and _TILE10 in cur and "AGPRs:" in line:
            n = int(line.split("AGPRs:", 1)[1].split()[0])
            if n < 256:
                bad.append((cur[:80], n))
    return bad


def _compile(src, flags, force, verbose, build_dir=BUILD_DIR):
    rel = os.path.relpath(src, CSRC).replace(os.sep, "_") if src.startswith(CSRC) else os.path.basename(src)
    obj = os.path.join(build_dir, rel + ".o")
    stamp = obj + ".hash"
    h = hashlib.sha256()
    with open(src, "rb") as fh:
        h.update(fh.read())
    h.update(" ".join(flags).encode())
    h.update(_deps_digest(src).encode())
    digest = h.hexdigest()
    if not force and os.path.exists(obj) and os.path.exists(stamp):
        with open(stamp) as fh:
            if fh.read().strip() == digest:
                return obj, False, ""
    cmd = [HIPCC, "-c", src, "-o", obj] + flags
    if src.endswith(".hip"):
        cmd = [HIPCC, "-x", "hip", "-c", src, "-o", obj] + flags
    gemm = os.path.basename(src).startswith("gemm")
    if gemm:
        cmd.append("-Rpass-analysis=kernel-resource-usage")
    if verbose:
        print(" ".join(cmd), flush=True)
    p = subprocess.run(cmd, capture_output=True, text=True)
    if p.returncode != 0:
        raise RuntimeError(f"compile failed: {src}\n{p.stdout}\n{p.stderr}")
    if gemm:
        bad = check_pinned_accumulators(p.stderr)
        if bad:
            os.remove(obj)
            raise RuntimeError(f"{src}: the 4-wave 256x256 GEMM tile lost its AGPR-pinned accumulators "
                               f"(needs 256 AGPRs; copies around every MFMA made it ~6x slower): {bad}")
        p = subprocess.CompletedProcess(p.args, 0, p.stdout, "\n".join(
            l for l in p.stderr.splitlines() if "kernel-resource-usage" not in l))
    with open(stamp, "w") as fh:
        fh.write(digest)
    return obj, True, p.stderr


def source_digest(debug=None):
    """sha256 over every file under csrc/ (path + content), the target arch and the debug flag:
    stamped into the built ``_C.so`` (``mift._C.source_hash()``) and checked by ``mift._ext`` at
    import, so a stale binary never runs silently against edited sources."""
    h = hashlib.sha256()
    for dp, _, fs in sorted(os.walk(CSRC)):
        for f in sorted(fs):
            if f.endswith((".hip", ".cpp", ".h", ".hpp", ".cuh", ".inc")):
                path = os.path.join(dp, f)
                h.update(os.path.relpath(path, CSRC).encode())
                with open(path, "rb") as fh:
                    h.update(fh.read())
    dbg = os.environ.get("MIFT_DEBUG") if debug is None else ("1" if debug else "")
    h.update(f"arch={ARCH};debug={1 if dbg else 0}".encode())
    return h.hexdigest()


def _write_build_info(build_dir=BUILD_DIR):
    path = os.path.join(build_dir, "build_info.cpp")
    text = ('// generated by mift/build.py: provenance stamp of this _C.so\n'
            f'extern "C" const char* mift_source_hash() {{ return "{source_digest()}"; }}\n')
    old = open(path).read() if os.path.exists(path) else None
    if old != text:
        with open(path, "w") as fh:
            fh.write(text)
    return path


def build(force=False, verbose=False, jobs=None):
    """Compile all sources and link ``_C.so``; returns the output path.

    ``MIFT_DEBUG=1`` compiles the device-side bounds checks (``MIFT_ASSERT`` in csrc/common.h)
    into ``_C_debug.so`` instead (load it with ``MIFT_EXT_SO=.../_C_debug.so``)."""
    debug = bool(os.environ.get("MIFT_DEBUG"))
    bdir = BUILD_DIR + ("_debug" if debug else "")
    os.makedirs(bdir, exist_ok=True)
    flags = _common_flags()
    srcs = _sources() + [_write_build_info(bdir)]
    jobs = jobs or min(16, max(1, (os.cpu_count() or 4)))
    objs, changed = [], False
    with cf.ThreadPoolExecutor(jobs) as ex:
        futs = [ex.submit(_compile, s, flags, force, verbose, bdir) for s in srcs]
        for f in futs:
            o, c, _ = f.result()
            objs.append(o)
            changed |= c
    out = OUT if not debug else os.path.join(HERE, "_C_debug.so")
    if changed or force or not os.path.exists(out):
        _, lib, _ = _torch_paths()
        tmp = out + ".tmp"
        cmd = [HIPCC, "-shared", "-fPIC", f"--offload-arch={ARCH}", "-o", tmp] + objs + [
            f"-L{lib}", "-lc10", "-lc10_hip", "-ltorch", "-ltorch_cpu", "-ltorch_hip", "-ltorch_python",
            f"-Wl,-rpath,{lib}"]
        if verbose:
            print(" ".join(cmd), flush=True)
        p = subprocess.run(cmd, capture_output=True, text=True)
        if p.returncode != 0:
            raise RuntimeError(f"link failed\n{p.stdout}\n{p.stderr}")
        os.replace(tmp, out)
    return out


def build_asan_loader(out_dir, verbose=False):
    """Host-only AddressSanitizer build of the native runtime (csrc/runtime/loader.cpp: the
    prefetching TokenLoader thread) as a stand-alone module ``_loader_asan`` (GPU
    sanitizers are not available, so the host code is checked on the CPU).  Run it under
    ``LD_PRELOAD=<libasan.so>`` (tests/test_loader_asan_cpu.py)."""
    os.makedirs(out_dir, exist_ok=True)
    inc, lib, abi = _torch_paths()
    py_inc = sysconfig.get_paths()["include"]
    mod = os.path.join(out_dir, "asan_module.cpp")
    with open(mod, "w") as fh:
        fh.write('#include <torch/extension.h>\nvoid mift_bind_runtime(pybind11::module& m);\n'
                 'PYBIND11_MODULE(_loader_asan, m) { mift_bind_runtime(m); }\n')
    so = os.path.join(out_dir, "_loader_asan.so")
    cmd = ["g++", "-O1", "-g", "-std=c++17", "-shared", "-fPIC", "-fsanitize=address", "-fno-omit-frame-pointer",
           f"-D_GLIBCXX_USE_CXX11_ABI={abi}", "-DTORCH_EXTENSION_NAME=_loader_asan", "-DTORCH_API_INCLUDE_EXTENSION_H",
           f"-I{py_inc}", "-o", so, os.path.join(CSRC, "runtime", "loader.cpp"), mod] + \
        [f"-isystem{i}" for i in inc] + \
        [f"-L{lib}", "-lc10", "-ltorch", "-ltorch_cpu", "-ltorch_python", f"-Wl,-rpath,{lib}"]
    if verbose:
        print(" ".join(cmd), flush=True)
    p = subprocess.run(cmd, capture_output=True, text=True)
    if p.returncode != 0:
        raise RuntimeError(f"asan loader build failed\n{p.stdout}\n{p.stderr}")
    return so


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--force", action="store_true")
    ap.add_argument("--verbose", action="store_true")
    ap.add_argument("--jobs", type=int, default=None)
    ap.add_argument("--debug", action="store_true", help="device bounds checks -> _C_debug.so")
    a = ap.parse_args(argv)
    if a.debug:
        os.environ["MIFT_DEBUG"] = "1"
    out = build(a.force, a.verbose, a.jobs)
    print(f"built {out}")


if __name__ == "__main__":
    sys.exit(main())
