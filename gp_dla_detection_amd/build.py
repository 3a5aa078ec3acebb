"""Build libgpdla.so in-tree with hipcc for gfx950 (no JIT cache, so the .so travels with the repo)."""
from __future__ import annotations

import os
import subprocess
import sys
from pathlib import Path

PKG = Path(__file__).resolve().parent
CSRC = PKG / "csrc"
SOURCES = ["kernels.hip", "kernels_i8.hip", "gemm_path.hip", "gemm_i8.hip", "gemm_f64.hip", "engine.hip", "objective.hip",
           "dla_samples.hip", "ingest.hip", "faddeeva_host.cpp"]
OUT = PKG / "libgpdla.so"


OBJ_DIR = PKG.parent / "build" / "obj"


def build(verbose: bool = False, force: bool = False, out: Path | None = None,
          defines: dict | None = None, jobs: int | None = None, define_only: set | None = None) -> Path:
    """Compile libgpdla.so (or a variant with -D``defines`` into ``out``, for A/B experiments;
    ``define_only`` limits the defines to those source files, the others come from the product build).

    Each translation unit is compiled to its own object in parallel (no cross-TU device code: every
    kernel is launched from the file that defines it), then linked; objects are reused while they
    are newer than their source and every header."""
    import hashlib
    from concurrent.futures import ThreadPoolExecutor
    OUT_ = Path(out) if out else OUT
    srcs = [CSRC / s for s in SOURCES]
    headers = list(CSRC.glob("*.h")) + [PKG.parent / "include" / "gpdla.h"]
    deps = srcs + headers
    if OUT_.exists() and not force and not defines and all(OUT_.stat().st_mtime >= d.stat().st_mtime for d in deps):
        return OUT_
    hipcc = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
    dflags = [f"-D{k}={v}" for k, v in sorted((defines or {}).items())]
    cflags = ["--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-c", "-Wno-unused-result", *dflags]
    # the object cache is keyed on everything that shapes an object besides its sources: the compiler
    # (path and mtime), the full flag list and this file (a changed recipe invalidates old objects)
    hipcc_path = Path(hipcc).resolve() if Path(hipcc).exists() else Path(hipcc)
    key = "\n".join([str(hipcc_path), str(hipcc_path.stat().st_mtime if hipcc_path.exists() else 0),
                     " ".join(cflags), str(Path(__file__).stat().st_mtime)])
    objdir = OBJ_DIR / hashlib.sha1(key.encode()).hexdigest()[:16]
    objdir.mkdir(parents=True, exist_ok=True)
    hdr_mtime = max(h.stat().st_mtime for h in headers)
    tmp_tag = f".{os.getpid()}.tmp"      # per-process temporaries: concurrent builds never share one

    base_flags = [f for f in cflags if f not in dflags]
    base_key = "\n".join([str(hipcc_path), str(hipcc_path.stat().st_mtime if hipcc_path.exists() else 0),
                          " ".join(base_flags), str(Path(__file__).stat().st_mtime)])
    base_dir = OBJ_DIR / hashlib.sha1(base_key.encode()).hexdigest()[:16]

    def compile_one(src: Path) -> Path:
        plain = define_only is not None and src.name not in define_only
        odir, flags = (base_dir, base_flags) if plain else (objdir, cflags)
        odir.mkdir(parents=True, exist_ok=True)
        obj = odir / (src.name + ".o")
        if not (force and not plain) and obj.exists() and obj.stat().st_mtime >= max(src.stat().st_mtime, hdr_mtime):
            return obj
        cmd = [hipcc, *flags, "-o", str(obj) + tmp_tag, str(src)]
        if verbose:
            print(" ".join(cmd), file=sys.stderr)
        subprocess.run(cmd, check=True, cwd=CSRC)
        Path(str(obj) + tmp_tag).replace(obj)
        return obj

    with ThreadPoolExecutor(max_workers=jobs or min(len(srcs), os.cpu_count() or 4)) as ex:
        objs = list(ex.map(compile_one, srcs))
    tmp = OUT_.with_name(OUT_.name + tmp_tag)
    cmd = [hipcc, "--offload-arch=gfx950", "-shared", "-fPIC", "-o", str(tmp), *map(str, objs)]
    if verbose:
        print(" ".join(cmd), file=sys.stderr)
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
