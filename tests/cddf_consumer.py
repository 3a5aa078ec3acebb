"""Run the reference's own consumer of processed_qsos_*.mat -- CDDF_analysis/calc_cddf.py's
DLACatalogue (calc_cddf.py:40-125, 224-247) -- on a file written by this package, and print what
it loaded as JSON.  Executed by tests/test_matv73.py with an interpreter that has h5py
(/opt/conda/bin/python3.9 in the build container); argv: reference CDDF_analysis dir,
processed file, DLA-samples file, SNR file.  Never runs on the GPU box (no /root/reference)."""
import json
import sys
import warnings

sys.dont_write_bytecode = True   # never write __pycache__ into the read-only reference tree

warnings.filterwarnings("ignore")
import numpy as np  # noqa: E402

if not hasattr(np, "bool"):
    np.bool = bool  # calc_cddf.py:84 uses the alias numpy 1.24 removed
import matplotlib  # noqa: E402

matplotlib.use("Agg")
sys.path.insert(0, sys.argv[1])
import calc_cddf  # noqa: E402

proc, samp, snrs = sys.argv[2:5]
cat = calc_cddf.DLACatalogue(processed_file=proc, sample_file=samp, raw_file=None, snrs_file=snrs, snr=-2)
extra = {}
for spec in range(len(cat.p_dla)):
    if spec not in cat.log_norm_like_cache and cat.p_dla[spec] > 0:
        # the on-demand path (calc_cddf.py:229-247) including its normalisation assert
        extra[spec] = cat._log_norm_like(spec).tolist()
print(json.dumps(dict(
    p_dla=cat.p_dla.tolist(), z_min=cat._z_min.tolist(), z_max=cat._z_max.tolist(),
    real_index=cat.real_index.tolist(), z_offsets=cat.z_offsets.tolist(), lnhi=cat.lnhi_vals.tolist(),
    log_norm_like={int(k): v.tolist() for k, v in cat.log_norm_like_cache.items()},
    log_norm_like_on_demand={int(k): v for k, v in extra.items()})))
