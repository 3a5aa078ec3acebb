"""Write tests/golden/speclite_fixture.fits with astropy (an independent FITS writer) for the
numpy FITS reader in gp_dla_detection_amd/ingest.py.  Run with an interpreter that has astropy
(/opt/conda/bin/python3.9 here).  The file has the DR12Q speclite layout read_spec.m reads
(primary HDU + binary table HDU 1: flux E, loglam E, ivar E, and_mask J, or_mask J, wdisp E,
sky E, model E; https://data.sdss.org/datamodel/files/BOSS_SPECTRO_REDUX/RUN2D/spectra/PLATE4/spec.html)
with synthetic values, plus an extra HDU 2 with unsigned / logical / string / vector columns."""
import os

import numpy as np

if not hasattr(np, "asscalar"):          # astropy 4.3 with numpy >= 1.23
    np.asscalar = lambda a: a.item()
if not hasattr(np, "alen"):
    np.alen = lambda a: len(a)
from astropy.io import fits

HERE = os.path.dirname(os.path.abspath(__file__))
rng = np.random.default_rng(11)
n = 500
loglam = (np.log10(3600.0) + 1e-4 * np.arange(n)).astype(np.float32)
flux = rng.normal(5, 1, n).astype(np.float32)
ivar = rng.uniform(0.5, 4, n).astype(np.float32)
ivar[rng.uniform(size=n) < 0.05] = 0
and_mask = rng.integers(0, 2 ** 30, n).astype(np.int32) & np.int32((1 << 23) | (1 << 22) | 1)
cols = [fits.Column("flux", "E", array=flux), fits.Column("loglam", "E", array=loglam),
        fits.Column("ivar", "E", array=ivar), fits.Column("and_mask", "J", array=and_mask),
        fits.Column("or_mask", "J", array=and_mask | 2), fits.Column("wdisp", "E", array=flux * 0 + 1),
        fits.Column("sky", "E", array=flux * 0), fits.Column("model", "E", array=flux)]
extra = [fits.Column("u16", "I", bzero=32768, array=np.arange(5, dtype=np.uint16) * 1000),
         fits.Column("flag", "L", array=np.array([True, False, True, True, False])),
         fits.Column("name", "6A", array=np.array(["abc", "de", "f", "ghijkl", ""])),
         fits.Column("vec", "3D", array=np.arange(15, dtype=np.float64).reshape(5, 3)),
         fits.Column("k64", "K", array=np.array([1, -2, 3, 2 ** 40, -(2 ** 40)], dtype=np.int64))]
hdus = fits.HDUList([fits.PrimaryHDU(np.zeros((3, 4), dtype=np.float32)),
                     fits.BinTableHDU.from_columns(cols), fits.BinTableHDU.from_columns(extra)])
hdus.writeto(os.path.join(HERE, "speclite_fixture.fits"), overwrite=True)
np.savez(os.path.join(HERE, "speclite_fixture.npz"), flux=flux, loglam=loglam, ivar=ivar, and_mask=and_mask)
print("wrote speclite_fixture.fits")
