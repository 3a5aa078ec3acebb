"""Build A/B variants of libgpdla into tools/variants/<name>.so (experiments only).

A variant is a set of -D defines for an experimental switch added to the sources for the length
of one A/B measurement (tools/ab_variants.sh, tools/prof_ab_ldl.sh run bench.py against each
variant through GPDLA_LIB).  Once measured, the losing code path is deleted from the product
sources; the outcomes of past experiments are recorded in DESIGN.md and under profiles/.
"""
import sys
from pathlib import Path
sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
from gp_dla_detection_amd.build import build

VARIANTS: dict = {
    "base": {},
    "ch50k": {"GPDLA_MAX_CHUNK": 50001},
    "ch25k": {"GPDLA_MAX_CHUNK": 25001},
    "ch16k": {"GPDLA_MAX_CHUNK": 16667},
    "bst_ex2": {"GPDLA_BST_EX": 2},
    "bst_ex8": {"GPDLA_BST_EX": 8},
    "cur": {"GPDLA_VARIANT_CUR": 1},     # the working tree as a variant (A/B against the in-tree build)
    "us45": {"GPDLA_BST_USPARE": "0.45f"},
    "us35": {"GPDLA_BST_USPARE": "0.35f"},
    "us40": {"GPDLA_BST_USPARE": "0.40f"},
    "us50": {"GPDLA_BST_USPARE": "0.50f"},
    "us25": {"GPDLA_BST_USPARE": "0.25f"},
    "us15": {"GPDLA_BST_USPARE": "0.15f"},
    "us55": {"GPDLA_BST_USPARE": "0.55f"},
    "us65": {"GPDLA_BST_USPARE": "0.65f"},
}
# variants whose defines only matter in some sources: the rest is linked from the product objects
ONLY = {n: {"gemm_i8.hip"} for n in ("cur", "us40", "us50", "us15", "us25", "us35", "us45", "us55", "us65")}

if __name__ == "__main__":
    names = sys.argv[1:] or list(VARIANTS)
    out = Path(__file__).resolve().parent / "variants"
    out.mkdir(exist_ok=True)
    for n in names:
        print(n, build(out=out / f"{n}.so", defines=VARIANTS[n] or {"GPDLA_VARIANT_BASE": 1}, force=True,
                       define_only=ONLY.get(n)))
