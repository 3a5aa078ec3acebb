"""Build libgpdla.so in-tree with hipcc for gfx950 (no JIT cache, so the .so travels with the repo)."""
from __future__ import annotations

import os
import subprocess
import sys
from pathlib import Path

PKG = Path(__file__).resolve().parent
CSRC = PKG / "csrc"
SOURCES = ["kernels.hip", "engine.hip", "faddeeva_host.cpp"]
OUT = PKG / "libgpdla.so"


def build(verbose: bool = False, force: bool = False) -> Path:
    srcs = [CSRC / s for s in SOURCES]
    deps = srcs + list(CSRC.glob("*.h")) + [PKG.parent / "include" / "gpdla.h"]
    if OUT.exists() and not force and all(OUT.stat().st_mtime >= d.stat().st_mtime for d in deps):
        return OUT
    hipcc = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
    cmd = [hipcc, "--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-shared",
           "-Wno-unused-result", "-o", str(OUT)] + [str(s) for s in srcs]
    if verbose:
        print(" ".join(cmd), file=sys.stderr)
    tmp = OUT.with_suffix(".so.tmp")
    cmd[cmd.index("-o") + 1] = str(tmp)
    subprocess.run(cmd, check=True, cwd=CSRC)
    tmp.replace(OUT)
    return OUT


if __name__ == "__main__":
    print(build(verbose=True, force="--force" in sys.argv))
