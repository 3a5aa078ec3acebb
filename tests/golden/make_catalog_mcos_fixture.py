"""Generate tests/golden/catalog_mcos.mat with libhdf5 (h5py; run with /opt/conda/bin/python3.9):
a catalog.mat in the shape build_catalogs.m saves (build_catalogs.m:50-53,117-119) -- numeric
columns, a uint8 filter_flags column, and containers.Map variables stored the way MATLAB stores
MCOS objects in v7.3 files (a uint32 handle dataset with MATLAB_class 'containers.Map' and
MATLAB_object_decode = 3, whose contents live in the '#subsystem#' group).  The handle and
subsystem payloads here are stand-in bytes: the test only needs a file whose objects this
package's reader cannot decode (run_preload_qsos must then not rewrite the file)."""
import os
import time

import h5py
import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))


def matlab_header():
    s = ("MATLAB 7.3 MAT-file, Platform: GLNXA64, Created on: "
         + time.strftime("%a %b %d %H:%M:%S %Y", time.gmtime(0)) + " HDF5 schema 1.00 .").encode()
    return s.ljust(116, b" ") + bytes(8) + (0x0200).to_bytes(2, "little") + b"IM"


def main():
    path = os.path.join(HERE, "catalog_mcos.mat")
    with h5py.File(path, "w", userblock_size=512, libver="earliest") as f:
        cols = dict(z_qsos=np.array([2.03, 2.5]), plates=np.array([4000.0, 4001.0]),
                    mjds=np.array([55000.0, 55001.0]), fiber_ids=np.array([12.0, 7.0]))
        for name, v in cols.items():
            d = f.create_dataset(name, data=v[None, :])          # MATLAB 2 x 1 -> HDF5 (1, 2)
            d.attrs["MATLAB_class"] = np.bytes_("double")
        d = f.create_dataset("filter_flags", data=np.array([[0, 2]], dtype=np.uint8))
        d.attrs["MATLAB_class"] = np.bytes_("uint8")
        for name in ("los_inds", "dla_inds", "z_dlas"):
            d = f.create_dataset(name, data=np.array([[3707764736], [2], [1], [1], [1], [1]], dtype=np.uint32))
            d.attrs["MATLAB_class"] = np.bytes_("containers.Map")
            d.attrs["MATLAB_object_decode"] = np.int32(3)
        g = f.create_group("#subsystem#")
        d = g.create_dataset("MCOS", data=np.arange(8, dtype=np.uint32)[None, :])
        d.attrs["MATLAB_class"] = np.bytes_("FileWrapper__")
    with open(path, "r+b") as fh:
        fh.write(matlab_header())


if __name__ == "__main__":
    main()
