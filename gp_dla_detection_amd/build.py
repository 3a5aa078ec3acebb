"""Build libgpdla.so in-tree with hipcc for gfx950 (no JIT cache, so the .so travels with the repo)."""
from __future__ import annotations

import os
import subprocess
import sys
from pathlib import Path

PKG = Path(__file__).resolve().parent
CSRC = PKG / "csrc"
SOURCES = ["kernels.hip", "kernels_i8.hip", "gemm_path.hip", "gemm_i8.hip", "gemm_f64.hip", "engine.hip", "objective.hip",
           "faddeeva_host.cpp"]
OUT = PKG / "libgpdla.so"


def build(verbose: bool = False, force: bool = False, out: Path | None = None,
          defines: dict | None = None) -> Path:
    """Compile libgpdla.so (or a variant with -D``defines`` into ``out``, for A/B experiments)."""
    OUT_ = Path(out) if out else OUT
    srcs = [CSRC / s for s in SOURCES]
    deps = srcs + list(CSRC.glob("*.h")) + [PKG.parent / "include" / "gpdla.h"]
    if OUT_.exists() and not force and not defines and all(OUT_.stat().st_mtime >= d.stat().st_mtime for d in deps):
        return OUT_
    hipcc = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
    cmd = [hipcc, "--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-shared",
           "-Wno-unused-result", "-o", str(OUT_)] + [f"-D{k}={v}" for k, v in (defines or {}).items()] \
        + [str(s) for s in srcs]
    if verbose:
        print(" ".join(cmd), file=sys.stderr)
    tmp = OUT_.with_suffix(".so.tmp")
    cmd[cmd.index("-o") + 1] = str(tmp)
    subprocess.run(cmd, check=True, cwd=CSRC)
    tmp.replace(OUT_)
    return OUT_


MEX_API = PKG.parent / "tests" / "support" / "mex_api"


def build_mex_mocks(verbose: bool = False) -> list[Path]:
    """Test support: each MATLAB gateway in matlab/ linked with the in-process MEX runtime of
    tests/support/mex_api/mex_mock.c into tests/support/mex_api/lib<gateway>_mock.so, so the tests
    drive the gateways' own code against libgpdla (no MATLAB here).  Host C only (gcc)."""
    import shutil
    cc = shutil.which("gcc") or shutil.which("cc")
    outs = []
    if not cc or not (PKG.parent / "matlab").is_dir():
        return outs
    for src in sorted((PKG.parent / "matlab").glob("*.c")):   # each includes matlab/mex_widen.h
        out = MEX_API / f"lib{src.stem}_mock.so"
        deps = [src, MEX_API / "mex_mock.c", MEX_API / "mex.h", PKG.parent / "include" / "gpdla.h",
                PKG.parent / "matlab" / "mex_widen.h"]
        if not (out.exists() and all(out.stat().st_mtime >= d.stat().st_mtime for d in deps)):
            cmd = [cc, "-std=c99", "-O1", "-Wall", "-fPIC", "-shared", f"-I{MEX_API}", f"-I{PKG.parent / 'include'}",
                   str(src), str(MEX_API / "mex_mock.c"), f"-L{PKG}", "-lgpdla",
                   "-Wl,-rpath,$ORIGIN/../../../gp_dla_detection_amd", "-o", str(out)]
            if verbose:
                print(" ".join(cmd), file=sys.stderr)
            subprocess.run(cmd, check=True)
        outs.append(out)
    return outs


if __name__ == "__main__":
    print(build(verbose=True, force="--force" in sys.argv))
