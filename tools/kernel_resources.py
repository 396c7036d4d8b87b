"""Print per-kernel VGPR/AGPR/spill/LDS/occupancy of a HIP source (hipcc -Rpass-analysis=kernel-resource-usage).

  python tools/kernel_resources.py gemm [filter]
"""
import os
import re
import subprocess
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from mift import build as B  # noqa: E402


def main(name, filt=""):
    src = os.path.join(os.path.dirname(B.__file__), "csrc", "kernels", name + ".hip")
    cmd = [B.HIPCC, "-x", "hip", "-c", src, "-o", "/tmp/_res.o", "-Rpass-analysis=kernel-resource-usage"] + \
        B._common_flags()
    out = subprocess.run(cmd, capture_output=True, text=True).stderr
    cur = None
    for line in out.splitlines():
        m = re.search(r"remark: (.*)", line)
        if not m:
            continue
        t = m.group(1)
        if t.startswith("Function Name:"):
            cur = t.split(":", 1)[1].strip()
            if filt in cur:
                print("\n" + cur[:150])
        elif cur and filt in cur and any(k in t for k in ("VGPRs", "AGPRs", "Spill", "Occupancy", "LDS Size")):
            print("   ", t)


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2] if len(sys.argv) > 2 else "")
