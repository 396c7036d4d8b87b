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


def _headers_digest():
    h = hashlib.sha256()
    for dp, _, fs in os.walk(CSRC):
        for f in sorted(fs):
            if f.endswith((".h", ".hpp", ".cuh", ".inc")):
                with open(os.path.join(dp, f), "rb") as fh:
                    h.update(f.encode())
                    h.update(fh.read())
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


def _compile(src, flags, hdr_digest, force, verbose):
    rel = os.path.relpath(src, CSRC).replace(os.sep, "_")
    obj = os.path.join(BUILD_DIR, rel + ".o")
    stamp = obj + ".hash"
    h = hashlib.sha256()
    with open(src, "rb") as fh:
        h.update(fh.read())
    h.update(" ".join(flags).encode())
    h.update(hdr_digest.encode())
    digest = h.hexdigest()
    if not force and os.path.exists(obj) and os.path.exists(stamp):
        with open(stamp) as fh:
            if fh.read().strip() == digest:
                return obj, False, ""
    cmd = [HIPCC, "-c", src, "-o", obj] + flags
    if src.endswith(".hip"):
        cmd = [HIPCC, "-x", "hip", "-c", src, "-o", obj] + flags
    if verbose:
        print(" ".join(cmd), flush=True)
    p = subprocess.run(cmd, capture_output=True, text=True)
    if p.returncode != 0:
        raise RuntimeError(f"compile failed: {src}\n{p.stdout}\n{p.stderr}")
    with open(stamp, "w") as fh:
        fh.write(digest)
    return obj, True, p.stderr


def build(force=False, verbose=False, jobs=None):
    """Compile all sources and link ``_C.so``; returns the output path."""
    os.makedirs(BUILD_DIR, exist_ok=True)
    flags = _common_flags()
    hdr = _headers_digest()
    srcs = _sources()
    jobs = jobs or min(16, max(1, (os.cpu_count() or 4)))
    objs, changed = [], False
    with cf.ThreadPoolExecutor(jobs) as ex:
        futs = [ex.submit(_compile, s, flags, hdr, force, verbose) for s in srcs]
        for f in futs:
            o, c, _ = f.result()
            objs.append(o)
            changed |= c
    if changed or force or not os.path.exists(OUT):
        _, lib, _ = _torch_paths()
        tmp = OUT + ".tmp"
        cmd = [HIPCC, "-shared", "-fPIC", f"--offload-arch={ARCH}", "-o", tmp] + objs + [
            f"-L{lib}", "-lc10", "-lc10_hip", "-ltorch", "-ltorch_cpu", "-ltorch_hip", "-ltorch_python",
            f"-Wl,-rpath,{lib}"]
        if verbose:
            print(" ".join(cmd), flush=True)
        p = subprocess.run(cmd, capture_output=True, text=True)
        if p.returncode != 0:
            raise RuntimeError(f"link failed\n{p.stdout}\n{p.stderr}")
        os.replace(tmp, OUT)
    return OUT


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--force", action="store_true")
    ap.add_argument("--verbose", action="store_true")
    ap.add_argument("--jobs", type=int, default=None)
    a = ap.parse_args(argv)
    out = build(a.force, a.verbose, a.jobs)
    print(f"built {out}")


if __name__ == "__main__":
    sys.exit(main())
