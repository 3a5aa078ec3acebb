"""Generate MATLAB-style v7.3 fixtures with libhdf5 (h5py) for the pure-numpy reader in
gp_dla_detection_amd/matv73.py.  Run with an interpreter that has h5py (here:
/opt/conda/bin/python3.9); the system python has none, which is why the product has its own
reader/writer.

The files follow the layout MATLAB's `save -v7.3` produces (512-byte MATLAB user block,
MATLAB_class attributes, column-major data with reversed dims, cells as object references into
#refs#, compressed variables as chunked datasets with the deflate filter, complex numbers as a
{real, imag} compound, logical as uint8 + MATLAB_int_decode) -- the shapes of the reference's
inputs: learned_qso_model_*.mat (learn_qso_model.m:103-123), dla_samples.mat
(generate_dla_samples.m:59-63) and preloaded_qsos.mat (preload_qsos.m:64-83).

Outputs: mat73_earliest.mat (superblock v0, symbol-table groups, chunked+deflate+shuffle),
mat73_latest.mat (superblock v3, v2 object headers, link messages, contiguous) and
mat73_expected.npz (the values, MATLAB-shaped, for the test to compare against).
"""
import os
import time

import h5py
import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))


def matlab_header():
    s = ("MATLAB 7.3 MAT-file, Platform: GLNXA64, Created on: "
         + time.strftime("%a %b %d %H:%M:%S %Y", time.gmtime(0)) + " HDF5 schema 1.00 .").encode()
    return s.ljust(116, b" ") + bytes(8) + (0x0200).to_bytes(2, "little") + b"IM"


def put(f, name, arr, cls, chunked, **extra):
    arr = np.asarray(arr)
    data = arr.T                                  # MATLAB r x c -> HDF5 (c, r)
    kw = dict(chunks=True, compression="gzip", shuffle=True) if chunked and data.size > 4 else {}
    d = f.create_dataset(name, data=data, **kw)
    d.attrs["MATLAB_class"] = np.bytes_(cls)
    for k, v in extra.items():
        d.attrs[k] = v
    return d


def write(path, libver, chunked, ncells):
    """One file; returns the MATLAB-shaped values it holds."""
    rng = np.random.default_rng(7)
    full = libver == "earliest"         # the libver="latest" file keeps <= 8 links per group
    with h5py.File(path, "w", userblock_size=512, libver=libver) as f:
        k = 6
        lam = np.arange(911.75, 1215.75 + 0.125, 0.25)
        mu = 1 + 0.1 * np.sin(lam / 10)
        M = rng.standard_normal((lam.size, k))
        put(f, "rest_wavelengths", lam[:, None], "double", chunked)
        put(f, "mu", mu[:, None], "double", chunked)
        put(f, "M", M, "double", chunked)
        put(f, "log_c_0", np.array([[np.log(0.1)]]), "double", False)
        z = (rng.standard_normal((4, 3)) + 1j * rng.standard_normal((4, 3)))
        cz = np.zeros(z.T.shape, dtype=[("real", "<f8"), ("imag", "<f8")])
        cz["real"], cz["imag"] = z.T.real, z.T.imag
        d = f.create_dataset("complex_var", data=cz)
        d.attrs["MATLAB_class"] = np.bytes_("double")
        exp = dict(rest_wavelengths=lam[:, None], mu=mu[:, None], M=M, log_c_0=np.array([[np.log(0.1)]]),
                   complex_var=z)
        if full:
            put(f, "num_quasars", np.array([[3]], dtype=np.int32), "int32", False)
            dr9 = rng.uniform(size=(1, 40)) < 0.5
            put(f, "in_dr9", dr9.astype(np.uint8), "logical", chunked, MATLAB_int_decode=np.int32(1))
            put(f, "release", np.frombuffer("dr12q".encode("utf-16-le"), "<u2")[None, :], "char", False,
                MATLAB_int_decode=np.int32(2))
            e = f.create_dataset("empty_var", data=np.array([0, 5], dtype=np.uint64))
            e.attrs["MATLAB_class"] = np.bytes_("double")
            e.attrs["MATLAB_empty"] = np.uint8(1)
            exp.update(num_quasars=np.array([[3]], dtype=np.int32), in_dr9=dr9)
        refs = f.create_group("#refs#")
        cells = []
        for i in range(ncells):            # 300 cells: a multi-level group B-tree in #refs#
            a = rng.standard_normal((int(rng.integers(1, 20)), 1))
            ds = put(refs, f"c{i:03d}", a, "double", chunked and i % 25 == 0)
            cells.append((ds.ref, a))
        cell = f.create_dataset("all_flux", data=np.array([[c[0] for c in cells]], dtype=h5py.ref_dtype))
        cell.attrs["MATLAB_class"] = np.bytes_("cell")
        exp.update(cell_lengths=np.array([c[1].shape[0] for c in cells]),
                   cell_concat=np.concatenate([c[1][:, 0] for c in cells]))
    with open(path, "r+b") as fh:
        fh.write(matlab_header())
    return exp


if __name__ == "__main__":
    exp = {}
    for tag, libver, chunked, ncells in (("earliest", "earliest", True, 300), ("latest", "latest", False, 5)):
        vals = write(os.path.join(HERE, f"mat73_{tag}.mat"), libver, chunked, ncells)
        exp.update({f"{tag}__{k}": v for k, v in vals.items()})
    np.savez(os.path.join(HERE, "mat73_expected.npz"), **exp)
    print("wrote", sorted(exp))
