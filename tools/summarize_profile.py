#!/usr/bin/env python3
"""Summarise a tools/profile.sh run (rocprofv3 CSVs) into profiles/<tag>_summary.json + .md.

Traffic accounting follows /opt/skills/guides/MI355X_MICROARCH.md (HBM section): FETCH_SIZE and
WRITE_SIZE are in KiB, collected in separate passes; on gfx950 FETCH_SIZE reports half the bytes
of a wide (16 B/lane) coalesced streaming read, so the read side is doubled.  Counts include
Infinity-Cache (MALL) hits.
"""
from __future__ import annotations

import collections
import csv
import json
import sys
from pathlib import Path


def load_counters(path):
    agg = collections.defaultdict(list)
    for r in csv.DictReader(open(path)):
        agg[(r["Kernel_Name"], r["Counter_Name"])].append(float(r["Counter_Value"]))
        if r["Counter_Name"] == "GRBM_GUI_ACTIVE":  # with the dispatch's own duration: the clock
            agg[(r["Kernel_Name"], "_dispatch_ns")].append(float(r["End_Timestamp"]) - float(r["Start_Timestamp"]))
    return agg


def main(src: str, tag: str, dst: str = "profiles"):
    src, dst = Path(src), Path(dst)
    dst.mkdir(exist_ok=True)
    stats = list(csv.DictReader(open(src / "trace" / "trace_kernel_stats.csv")))
    fetch = load_counters(src / "fetch" / "fetch_counter_collection.csv")
    write = load_counters(src / "write" / "write_counter_collection.csv")
    sq = load_counters(src / "sq" / "sq_counter_collection.csv")
    bench = json.loads((src / "bench_trace.json").read_text().strip().splitlines()[-1])
    out = {"tag": tag, "bench_under_trace": {k: bench[k] for k in ("value", "unit", "ms_per_step", "kernel_ms")},
           "kernels": []}
    for row in stats:
        name = row["Name"]
        short = name.replace("(anonymous namespace)::", "")
        ent = {"kernel": short, "calls": int(row["Calls"]), "avg_ms": float(row["AverageNs"]) / 1e6,
               "pct": float(row["Percentage"])}
        key = next((k for k in fetch if k[0] == name and k[1] == "FETCH_SIZE"), None)
        wkey = next((k for k in write if k[0] == name and k[1] == "WRITE_SIZE"), None)
        if key and wkey:
            f_kib = sum(fetch[key]) / len(fetch[key])
            w_kib = sum(write[wkey]) / len(write[wkey])
            ent["fetch_size_kib"] = f_kib
            ent["write_size_kib"] = w_kib
            ent["hbm_bytes_per_launch"] = (2 * f_kib + w_kib) * 1024
            ent["hbm_gbs"] = ent["hbm_bytes_per_launch"] / (ent["avg_ms"] * 1e-3) / 1e9
        for cn in ("SQ_INSTS_VALU", "SQ_INSTS_MFMA", "SQ_INSTS_LDS", "SQ_WAVES", "SQ_WAVE_CYCLES", "SQ_BUSY_CYCLES",
                   "GRBM_GUI_ACTIVE"):
            k = (name, cn)
            if k in sq:
                ent[cn] = sum(sq[k]) / len(sq[k])
        # effective clock (MI355X_MICROARCH.md, DVFS give-back: GRBM_GUI_ACTIVE / 8 XCDs / dispatch time;
        # reads high below ~0.3 ms) and, for f64-MFMA kernels, the share of the SIMDs' DP-pipe cycles
        # their instructions need (v_mfma_f64_4x4x4_4b 16 cycles, other VALU 4; gfx950 counts MFMAs
        # inside SQ_INSTS_VALU)
        kd = (name, "_dispatch_ns")
        if kd in sq and "GRBM_GUI_ACTIVE" in ent:
            ns = sum(sq[kd]) / len(sq[kd])
            ent["eff_clock_ghz"] = ent["GRBM_GUI_ACTIVE"] / 8 / ns
            if "likelihood_kernel" in short and all(c in ent for c in ("SQ_INSTS_VALU", "SQ_INSTS_MFMA")):
                need = 16 * ent["SQ_INSTS_MFMA"] + 4 * (ent["SQ_INSTS_VALU"] - ent["SQ_INSTS_MFMA"])
                ent["dp_pipe_busy_frac"] = need / (1024 * ent["GRBM_GUI_ACTIVE"] / 8)
        out["kernels"].append(ent)
    # per batch (one gpdla_engine_process batch = one prep launch): the HBM bytes of every kernel
    # with counters, for the panel paths whose "launch" is a batch of many kernels
    preps = [e for e in out["kernels"] if e["kernel"].startswith("void gpdla::prep_kernel")]
    if preps:
        nb = sum(e["calls"] for e in preps)
        tot = sum(e["hbm_bytes_per_launch"] * e["calls"] for e in out["kernels"] if "hbm_bytes_per_launch" in e)
        out["per_batch"] = {"batches": nb, "hbm_bytes_per_batch": tot / nb,
                            "kernel_ms_per_batch": sum(e["avg_ms"] * e["calls"] for e in out["kernels"]) / nb}
    (dst / f"{tag}_summary.json").write_text(json.dumps(out, indent=1))
    lines = [f"# rocprofv3 summary `{tag}`", "",
             f"bench under trace: {bench['value']:.4g} {bench['unit']}, {bench['ms_per_step']:.2f} ms/step", "",
             "| kernel | calls | avg ms | % | HBM GB/launch (2*FETCH+WRITE) | HBM GB/s | VALU/wave | MFMA/wave | LDS/wave | clock GHz |",
             "|---|---|---|---|---|---|---|---|---|---|"]
    for e in out["kernels"]:
        w = e.get("SQ_WAVES") or 0
        per = lambda c: f"{e[c] / w:.0f}" if w and c in e else "-"
        gb = f"{e['hbm_bytes_per_launch'] / 1e9:.3f}" if "hbm_bytes_per_launch" in e else "-"
        gbs = f"{e['hbm_gbs']:.0f}" if "hbm_gbs" in e else "-"
        lines.append(f"| {e['kernel']} | {e['calls']} | {e['avg_ms']:.3f} | {e['pct']:.2f} | {gb} | {gbs} | "
                     f"{per('SQ_INSTS_VALU')} | {per('SQ_INSTS_MFMA')} | {per('SQ_INSTS_LDS')} | "
                     f"{e['eff_clock_ghz']:.2f} |" if "eff_clock_ghz" in e else
                     f"| {e['kernel']} | {e['calls']} | {e['avg_ms']:.3f} | {e['pct']:.2f} | {gb} | {gbs} | "
                     f"{per('SQ_INSTS_VALU')} | {per('SQ_INSTS_MFMA')} | {per('SQ_INSTS_LDS')} | - |")
        if "dp_pipe_busy_frac" in e:
            lines.append(f"|  ↳ DP pipe: its f64 MFMA + VALU issue needs {100 * e['dp_pipe_busy_frac']:.1f}% of the "
                         f"SIMDs' cycles at the measured clock | | | | | | | | | |")
    if "per_batch" in out:
        pb = out["per_batch"]
        lines += ["", f"per batch ({pb['batches']} batches): {pb['hbm_bytes_per_batch'] / 1e9:.2f} GB of HBM traffic, "
                      f"{pb['kernel_ms_per_batch']:.2f} ms of kernel time"]
    (dst / f"{tag}_summary.md").write_text("\n".join(lines) + "\n")
    print("\n".join(lines))


if __name__ == "__main__":
    main(*sys.argv[1:])
