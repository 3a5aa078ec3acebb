"""``set_parameters`` mirror (set_parameters.m:1-92).

The reference's set_parameters is a MATLAB *script* that drops variables and lambdas into the
caller's workspace.  Here the same names are module constants, and ``set_parameters()`` returns
a frozen object carrying them (plus the redshift helpers), so a port of a MATLAB session reads::

    params = set_parameters()
    process_qsos(..., params=params)
"""
from __future__ import annotations

import dataclasses
import math

import numpy as np

# physical constants (set_parameters.m:5-8)
LYA_WAVELENGTH = 1215.6701
LYB_WAVELENGTH = 1025.7223
LYMAN_LIMIT = 911.7633
SPEED_OF_LIGHT = 299792458


def kms_to_z(kms):  # set_parameters.m:11
    return (kms * 1000) / SPEED_OF_LIGHT


def emitted_wavelengths(observed_wavelengths, z):  # set_parameters.m:14-15
    return observed_wavelengths / (1 + z)


def observed_wavelengths(emitted_wavelengths, z):  # set_parameters.m:17-18
    return emitted_wavelengths * (1 + z)


# file loading / preprocessing (set_parameters.m:21-30)
LOADING_MIN_LAMBDA = 910
LOADING_MAX_LAMBDA = 1217
Z_QSO_CUT = 2.15
MIN_NUM_PIXELS = 200
NORMALIZATION_MIN_LAMBDA = 1310
NORMALIZATION_MAX_LAMBDA = 1325

# null model (set_parameters.m:33-37)
MIN_LAMBDA = 911.75
MAX_LAMBDA = 1215.75
DLAMBDA = 0.25
K = 20
MAX_NOISE_VARIANCE = 1 ** 2

# optimisation initial values (set_parameters.m:40-45)
INITIAL_C_0 = 0.1
INITIAL_TAU_0 = 0.0023
INITIAL_BETA = 3.65

# DLA sample parameters (set_parameters.m:48-53)
NUM_DLA_SAMPLES = 10000
ALPHA = 0.9
UNIFORM_MIN_LOG_NHI = 20.0
UNIFORM_MAX_LOG_NHI = 23.0
FIT_MIN_LOG_NHI = 20.0
FIT_MAX_LOG_NHI = 22.0

# prior (set_parameters.m:56)
PRIOR_Z_QSO_INCREASE = kms_to_z(30000)

# instrumental broadening (set_parameters.m:59-60); must equal voigt.c:229's width
WIDTH = 3
PIXEL_SPACING = 1e-4

# absorber range and model (set_parameters.m:63-73)
NUM_LINES = 3
MAX_Z_CUT = kms_to_z(3000)
MIN_Z_CUT = kms_to_z(3000)


def max_z_dla(wavelengths, z_qso):  # set_parameters.m:66-67
    return (np.max(wavelengths) / LYA_WAVELENGTH - 1) - MAX_Z_CUT


def min_z_dla(wavelengths, z_qso):  # set_parameters.m:70-73
    return max(np.min(wavelengths) / LYA_WAVELENGTH - 1,
               observed_wavelengths(LYMAN_LIMIT, z_qso) / LYA_WAVELENGTH - 1 + MIN_Z_CUT)


# directories (set_parameters.m:76-89)
BASE_DIRECTORY = "data"


def distfiles_directory(release):
    return f"{BASE_DIRECTORY}/{release}/distfiles"


def spectra_directory(release):
    return f"{BASE_DIRECTORY}/{release}/spectra"


def processed_directory(release):
    return f"{BASE_DIRECTORY}/{release}/processed"


def dla_catalog_directory(name):
    return f"{BASE_DIRECTORY}/dla_catalogs/{name}/processed"


@dataclasses.dataclass(frozen=True)
class Parameters:
    """The hot-path knobs of set_parameters.m, as one frozen value."""
    k: int = K
    num_dla_samples: int = NUM_DLA_SAMPLES
    num_lines: int = NUM_LINES
    width: int = WIDTH
    pixel_spacing: float = PIXEL_SPACING
    min_lambda: float = MIN_LAMBDA
    max_lambda: float = MAX_LAMBDA
    dlambda: float = DLAMBDA
    lya_wavelength: float = LYA_WAVELENGTH
    lyman_limit: float = LYMAN_LIMIT
    max_z_cut: float = MAX_Z_CUT
    min_z_cut: float = MIN_Z_CUT
    prior_z_qso_increase: float = PRIOR_Z_QSO_INCREASE
    # "reference": reproduce process_qsos.m:180,189 (absorption(1:n) of the m in-range values);
    # "unmasked": pair each unmasked pixel with its own profile value (the evident intent).
    absorption_mode: str = "reference"

    def __post_init__(self):
        if self.width != 3:
            raise ValueError("width must equal voigt.c:229's compiled-in width (3)")
        if not 1 <= self.num_lines <= 31:
            raise ValueError("num_lines must be in [1, 31] (voigt.c:16)")
        if self.absorption_mode not in ("reference", "unmasked"):
            raise ValueError("absorption_mode must be 'reference' or 'unmasked'")
        if self.k < 1:
            raise ValueError("k must be >= 1")


def set_parameters(**overrides) -> Parameters:
    return Parameters(**overrides)


LOG_2PI = 1.83787706640934534  # log_mvnpdf_low_rank.m:7
assert abs(LOG_2PI - math.log(2 * math.pi)) < 1e-15
