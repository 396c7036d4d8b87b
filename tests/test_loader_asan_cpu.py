"""Host AddressSanitizer run of the native runtime (csrc/runtime/loader.cpp).

The prefetching TokenLoader (a C++ worker thread writing pinned-memory batches into a bounded
queue) is built stand-alone with ``-fsanitize=address`` (mift.build.build_asan_loader) and driven
through early stops, restarts, resumes mid-epoch, tiny queues and a bad index, in a child Python
process with libasan preloaded.  Any heap / use-after-free / race-induced overflow aborts it."""
import os
import subprocess
import sys

import pytest

from mift import build as B

DRIVER = r'''
import sys, torch
sys.path.insert(0, sys.argv[1])
import _loader_asan as L
N, S = 37, 24
ids = torch.randint(0, 500, (N, S), dtype=torch.int32)
lens = torch.randint(1, S + 1, (N,), dtype=torch.int32)
for prefetch in (1, 2, 7):
    ld = L.TokenLoader(ids, lens, 499, 5, prefetch, False)
    order = torch.randperm(N)
    ld.start(order, 0)
    n = 0
    while True:
        b = ld.next()
        if not b:
            break
        n += b[0].shape[0]
        assert b[1].sum(1).le(S).all()
    assert n == N, n
    ld.start(order, 3)          # resume mid-epoch (restart while the old worker is gone)
    b = ld.next()
    assert b and b[0].shape[0] == 5
    ld.start(order, 0)          # restart while the worker is still producing
    ld.stop()
    del ld                      # destructor joins the thread
bad = L.TokenLoader(ids, lens, 499, 4, 2, False)
try:
    bad.start(torch.tensor([0, N + 3]), 0)
    raise SystemExit("out-of-range index accepted")
except RuntimeError:
    pass
print("ASAN-DRIVER-OK")
'''


def test_token_loader_under_asan(tmp_path):
    asan = subprocess.run(["gcc", "-print-file-name=libasan.so"], capture_output=True, text=True).stdout.strip()
    if not asan or not os.path.exists(asan):
        pytest.skip("libasan not available")
    so = B.build_asan_loader(str(tmp_path))
    # libstdc++ preloaded next to libasan: python itself does not link it, and ASan's __cxa_throw
    # interceptor must resolve the real symbol at startup (the loader reports errors by throwing)
    cxx = subprocess.run(["gcc", "-print-file-name=libstdc++.so.6"], capture_output=True, text=True).stdout.strip()
    env = dict(os.environ, LD_PRELOAD=f"{asan} {cxx}", ASAN_OPTIONS="detect_leaks=0:abort_on_error=1:halt_on_error=1")
    p = subprocess.run([sys.executable, "-c", DRIVER, os.path.dirname(so)], env=env, capture_output=True, text=True,
                       timeout=600)
    assert "AddressSanitizer" not in p.stderr, p.stderr[-4000:]
    assert p.returncode == 0 and "ASAN-DRIVER-OK" in p.stdout, (p.stdout[-2000:], p.stderr[-4000:])
