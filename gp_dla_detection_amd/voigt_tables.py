"""Lyman-series constants on the Python side (used only by the synthetic-data generator to
inject DLAs).  Same values as csrc/lyman_series.h (voigt.c:22,31-64,146,151-220)."""
import numpy as np

C_CGS = 2.99792458e10
SIGMA = 9.08537121627923800e+05
TRANSITION_WAVELENGTHS = np.array([1.2156701e-05, 1.0257223e-05, 9.725368e-06])
LEADING_CONSTANTS = np.array([1.34347262962625339e-07, 2.15386482180851912e-08, 7.48525170087141461e-09])
LORENTZ_GAMMAS = np.array([6.06075804241938613e+02, 1.54841462408931704e+02, 6.28964942715328164e+01])
