#!/usr/bin/env python
"""Build an EXPERIMENTAL copy of the extension from ``.wip/csrc`` into ``.wip/_C_exp.so``.

Kernel experiments are edited in ``.wip/csrc`` (a copy of the package's csrc/ tree, not tracked by git)
so the in-tree ``_C.so`` and its sources stay consistent while a GPU call is queued (the GPU box
snapshots the tree only when it starts, and the loader refuses a ``_C.so`` whose stamp does not
match csrc/).  Load the experimental build with ``MIFT_EXT_SO=.wip/_C_exp.so`` (no provenance check
on an explicit path); A/B it against the in-tree build in one process with tools/ab_ext.py.

  python tools/build_exp.py [--init] [--jobs N]
"""
import argparse
import concurrent.futures as cf
import os
import shutil
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from mift import build as B  # noqa: E402

WIP = os.path.join(ROOT, ".wip")
SRC = os.path.join(WIP, "csrc")
BDIR = os.path.join(WIP, "build")
OUT = os.path.join(WIP, "_C_exp.so")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--init", action="store_true", help="(re)copy the package csrc/ into .wip/csrc")
    ap.add_argument("--jobs", type=int, default=8)
    ap.add_argument("--only", default=None, help="comma list of source basenames to rebuild (others cached)")
    a = ap.parse_args()
    if a.init or not os.path.isdir(SRC):
        shutil.rmtree(SRC, ignore_errors=True)
        shutil.copytree(B.CSRC, SRC)
    os.makedirs(BDIR, exist_ok=True)
    flags = [f for f in B._common_flags() if not f.startswith(f"-I{B.CSRC}")] + [f"-I{SRC}"]
    srcs = []
    for dp, _, fs in os.walk(SRC):
        for f in sorted(fs):
            if f.endswith((".hip", ".cpp")):
                srcs.append(os.path.join(dp, f))
    info = os.path.join(BDIR, "build_info.cpp")
    with open(info, "w") as fh:
        fh.write('extern "C" const char* mift_source_hash() { return "experimental"; }\n')
    srcs.append(info)
    with cf.ThreadPoolExecutor(a.jobs) as ex:
        objs = [o for o, _, _ in ex.map(lambda s: B._compile(s, flags, False, False, BDIR), srcs)]
    _, lib, _ = B._torch_paths()
    cmd = [B.HIPCC, "-shared", "-fPIC", f"--offload-arch={B.ARCH}", "-o", OUT + ".tmp"] + objs + [
        f"-L{lib}", "-lc10", "-lc10_hip", "-ltorch", "-ltorch_cpu", "-ltorch_hip", "-ltorch_python",
        f"-Wl,-rpath,{lib}"]
    p = subprocess.run(cmd, capture_output=True, text=True)
    if p.returncode:
        raise SystemExit(p.stderr)
    os.replace(OUT + ".tmp", OUT)
    print(f"built {OUT}")


if __name__ == "__main__":
    main()
