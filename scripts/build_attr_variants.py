#!/usr/bin/env python3
"""Timing-only attribution builds of fused5 (wrong numerics; never the
production library): libbdx_hip_<name>.so from a scratch copy of the sources.

  d1  no contractions: the x / z / y passes are replaced by a scaled copy of
      the staged input (loads, staging, p / x stores and the gather remain)
  d4  no next-layer loads (the staging stores remain, of zeros)
  d6  d4 and no gather stores

  python scripts/build_attr_variants.py d1 d4 d6
"""
import shutil
import subprocess
import sys
import tempfile
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]


def patch(src: str, name: str) -> str:
    if name in ("d1",):
        a = src.index("    // ------------------------------------------------ x pass: lane (j, k) = (la, lb)")
        b = src.index("    // element dot p_e . (A_e p_e)")
        src = src[:a] + ("    T ye[ND];\n#pragma unroll\n    for (int j = 0; j < ND; ++j)\n"
                         "      ye[j] = ucell[la * PLP + j * DZP + lb] * G00;\n") + src[b:]
    if name in ("d4", "d6"):
        old = "        if (last || !(m & (1 << 21))) continue;\n"
        assert src.count(old) == 2, src.count(old)
        src = src.replace(old, "        continue;\n")
        tail = "\n        if (BDX_OOB(lnext + st_goff[k], A.vsize, \"f5 prefetch\")) continue;"
        old = "      if (!last && (st_meta[k] & kValid)) {" + tail
        assert src.count(old) == 1
        src = src.replace(old, "      if (false) {" + tail)
    if name == "d6":
        old = "          if (red || (pl == P && !glast)) continue;"
        assert src.count(old) == 1
        src = src.replace(old, "          continue;")
    return src


def main(names):
    for name in names:
        tmp = Path(tempfile.mkdtemp())
        shutil.copytree(ROOT / "benchmark_dolfinx_amd", tmp / "benchmark_dolfinx_amd")
        for so in (tmp / "benchmark_dolfinx_amd" / "ops").glob("*.so*"):
            so.unlink()
        h = tmp / "benchmark_dolfinx_amd" / "csrc" / "hip" / "lap_fused5.h"
        h.write_text(patch(h.read_text(), name))
        subprocess.run([sys.executable, "-m", "benchmark_dolfinx_amd.ops.build", "--hip", "-j", "8"],
                       cwd=tmp, check=True, capture_output=True)
        shutil.copy(tmp / "benchmark_dolfinx_amd" / "ops" / "libbdx_hip.so",
                    ROOT / "benchmark_dolfinx_amd" / "ops" / f"libbdx_hip_{name}.so")
        shutil.rmtree(tmp)
        print("built", name)


if __name__ == "__main__":
    main(sys.argv[1:])
