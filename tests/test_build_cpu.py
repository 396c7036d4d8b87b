"""Build provenance and debug builds (VERDICT r1 hygiene):

* the in-tree ``_C.so`` carries the sha256 of the csrc/ tree it was built from, and the loader
  refuses a binary whose stamp does not match the sources next to it;
* the debug configuration (``-DMIFT_DEBUG=1``: device-side ``MIFT_ASSERT`` bounds checks)
  compiles for gfx950.
"""
import os
import subprocess
import sys

import pytest

from mift import build as B

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_extension_is_stamped_with_current_sources():
    import mift
    if not os.path.exists(B.OUT):
        pytest.skip("extension not built")
    assert mift.kernels_available(), mift._ext.error()
    assert mift._ext.require().source_hash() == B.source_digest(debug=False)


def test_stale_extension_is_refused():
    from mift import _ext

    class Fake:
        @staticmethod
        def source_hash():
            return "0" * 64

    with pytest.raises(ImportError, match="stale extension"):
        _ext._check_provenance(Fake, os.path.join(B.HERE, "_C.so"), B.HERE)


def test_digest_tracks_sources(tmp_path, monkeypatch):
    d0 = B.source_digest(debug=False)
    assert d0 != B.source_digest(debug=True)
    fake = tmp_path / "csrc"
    (fake / "kernels").mkdir(parents=True)
    (fake / "kernels" / "a.hip").write_text("// a\n")
    monkeypatch.setattr(B, "CSRC", str(fake))
    d1 = B.source_digest(debug=False)
    (fake / "kernels" / "a.hip").write_text("// b\n")
    assert B.source_digest(debug=False) != d1


def test_debug_kernel_build_compiles(tmp_path):
    src = os.path.join(B.CSRC, "kernels", "elementwise.hip")
    cmd = [B.HIPCC, "-x", "hip", "-c", src, "-o", str(tmp_path / "e.o")] + B._common_flags() + ["-DMIFT_DEBUG=1"]
    p = subprocess.run(cmd, capture_output=True, text=True, timeout=600)
    assert p.returncode == 0, p.stderr[-2000:]


def test_pinned_accumulator_check_parses_resource_remarks():
    """build.py refuses a GEMM object whose 4-wave 256x256 tile has fewer than 256 AGPRs (its
    accumulators copied between register files around every MFMA: the round-6 79 -> 514 ms slip)."""
    from mift import build as B
    k10 = "_ZN12_GLOBAL__N_114gemm_nt_kernelIDF16_Li256ELi256ELi2ELi2ELi1ELb0ELi0ELi64EEEvPKT_"
    k8 = "_ZN12_GLOBAL__N_114gemm_nt_kernelIDF16_Li256ELi256ELi4ELi2ELi3ELb0ELi0ELi64EEEvPKT_"
    rem = lambda k, a: (f"gemm_impl.h:1:1: remark: {k}: Function Name: {k} [-Rpass-analysis=kernel-resource-usage]\n"
                        f"gemm_impl.h:1:1: remark: {k}:     VGPRs: 256 [-Rpass-analysis=kernel-resource-usage]\n"
                        f"gemm_impl.h:1:1: remark: {k}:     AGPRs: {a} [-Rpass-analysis=kernel-resource-usage]\n")
    assert B.check_pinned_accumulators(rem(k10, 256) + rem(k8, 0)) == []
    bad = B.check_pinned_accumulators(rem(k8, 0) + rem(k10, 65))
    assert len(bad) == 1 and bad[0][1] == 65
