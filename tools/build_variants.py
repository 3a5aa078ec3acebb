"""Build A/B variants of libgpdla into tools/variants/<name>.so (experiments only)."""
import sys
from pathlib import Path
sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
from gp_dla_detection_amd.build import build

VARIANTS = {
    "f1_e1": dict(GPDLA_SCHED_FENCE=1, GPDLA_FAST_EXP=1),
    "f1_e0": dict(GPDLA_SCHED_FENCE=1, GPDLA_FAST_EXP=0),
    "f0_e1": dict(GPDLA_SCHED_FENCE=0, GPDLA_FAST_EXP=1),
    "f1_w1": dict(GPDLA_SCHED_FENCE=1, GPDLA_WAVES_PER_EU=1),
    "f0_w1": dict(GPDLA_SCHED_FENCE=0, GPDLA_WAVES_PER_EU=1),
    "epi_lds": dict(GPDLA_LDS_EPILOGUE=1),
    "epi_global": dict(GPDLA_LDS_EPILOGUE=0),
    "m1s1": dict(GPDLA_MAGIC_RINT=1, GPDLA_SHARED_RCP=1),
    "m1s0": dict(GPDLA_MAGIC_RINT=1, GPDLA_SHARED_RCP=0),
    "m0s0": dict(GPDLA_MAGIC_RINT=0, GPDLA_SHARED_RCP=0),
    "far1": dict(GPDLA_FAR_WING=1),
    "far0": dict(GPDLA_FAR_WING=0),
    "i8pipe1": dict(I8_PIPELINE=1),
    "i8pipe0": dict(I8_PIPELINE=0),
    "gemm_pf1": dict(GPDLA_GEMM_I8_REGPF=1),
    "gemm_pf0": dict(GPDLA_GEMM_I8_REGPF=0),
    "ldl_reg": dict(GPDLA_LDL_CYCLIC=0),
    "ldl_cyc_stage": dict(GPDLA_LDL_CYCLIC=1, GPDLA_LDL_GATHER=0),
    "ldl_cyc_gather": dict(GPDLA_LDL_CYCLIC=1, GPDLA_LDL_GATHER=1),
    "ldl_ovl0": dict(GPDLA_LDL_OVERLAP=0),
    "ldl_ovl1": dict(GPDLA_LDL_OVERLAP=1),
}
if __name__ == "__main__":
    names = sys.argv[1:] or list(VARIANTS)
    out = Path(__file__).resolve().parent / "variants"
    out.mkdir(exist_ok=True)
    for n in names:
        print(n, build(out=out / f"{n}.so", defines=VARIANTS[n], force=True))
