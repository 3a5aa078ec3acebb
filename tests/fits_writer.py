"""Minimal FITS writer for tests: a primary HDU without data plus one binary table with the DR12Q
speclite columns read_spec.m reads (flux E, loglam E, ivar E, and_mask J).  Test helper only; the
product reads FITS (gp_dla_detection_amd/ingest.py) and never writes it."""
import numpy as np


def _card(key, value=None, comment=""):
    if value is None:
        return f"{key:<80}"[:80]
    if isinstance(value, bool):
        v = "T" if value else "F"
        s = f"{key:<8}= {v:>20}"
    elif isinstance(value, (int, np.integer)):
        s = f"{key:<8}= {int(value):>20}"
    else:
        s = f"{key:<8}= '{value:<8}'"
    if comment:
        s += f" / {comment}"
    return f"{s:<80}"[:80]


def _block(cards):
    raw = "".join(cards + [_card("END")])
    raw += " " * (-len(raw) % 2880)
    return raw.encode("ascii")


def write_speclite(path, flux, loglam, ivar, and_mask):
    n = len(flux)
    cols = [("flux", "E", ">f4", flux), ("loglam", "E", ">f4", loglam), ("ivar", "E", ">f4", ivar),
            ("and_mask", "J", ">i4", and_mask)]
    row = np.zeros(n, dtype=[(c[0], c[2]) for c in cols])
    for name, _, dt, arr in cols:
        row[name] = np.asarray(arr).astype(dt)
    primary = _block([_card("SIMPLE", True), _card("BITPIX", 8), _card("NAXIS", 0), _card("EXTEND", True)])
    hdr = [_card("XTENSION", "BINTABLE"), _card("BITPIX", 8), _card("NAXIS", 2),
           _card("NAXIS1", row.dtype.itemsize), _card("NAXIS2", n), _card("PCOUNT", 0), _card("GCOUNT", 1),
           _card("TFIELDS", len(cols))]
    for i, (name, form, _, _) in enumerate(cols, 1):
        hdr += [_card(f"TTYPE{i}", name), _card(f"TFORM{i}", form)]
    data = row.tobytes()
    data += b"\0" * (-len(data) % 2880)
    with open(path, "wb") as f:
        f.write(primary + _block(hdr) + data)
