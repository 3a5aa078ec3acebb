#!/usr/bin/env python3
"""Summarise a tools/profile_ingest.sh run: per ingest kernel, launches, time, algorithmic bytes
(tools/bench_ingest.py's accounting) over kernel time against the 8 TB/s HBM peak, and the PMC bytes
per launch (FETCH_SIZE doubled for gfx950's wide streaming reads, WRITE_SIZE as is; both KiB;
MI355X_MICROARCH.md's HBM section; they include Infinity-Cache hits).

    python3 tools/summarize_ingest.py <profile_ingest.sh dir> [summary.json] > summary.md"""
import collections
import csv
import json
import sys
from pathlib import Path

HBM_PEAK_GBS = 8000.0


def counters(path, name):
    agg = collections.defaultdict(float)
    for r in csv.DictReader(open(path)):
        if r["Counter_Name"] == name:
            agg[r["Kernel_Name"]] += float(r["Counter_Value"])
    return agg


def main(src, json_out=None):
    src = Path(src)
    rec = {"source": str(src), "kernels": {}}
    bench = json.loads((src / "bench_trace.json").read_text())
    pq = bench["preload_qsos_dr12q"]
    warm = pq["warmup"]
    alg = {"preload_scan_kernel": 12 * (pq["pixels_in"] + warm["pixels_in"]),
           "preload_write_kernel": 29 * (pq["pixels_out"] + warm["pixels_out"])}
    trace = list(csv.DictReader(open(src / "trace" / "trace_kernel_stats.csv")))
    fetch = counters(src / "fetch" / "fetch_counter_collection.csv", "FETCH_SIZE")
    write = counters(src / "write" / "write_counter_collection.csv", "WRITE_SIZE")
    print(f"# Ingest kernels over the DR12Q count ({pq['spectra']:,} spectra, {pq['batches']} batches + 1 warm-up launch)\n")
    print(f"{pq['pixels_in']:,} input pixels, {pq['pixels_out']:,} selected; host wall {pq['wall_s']:.2f} s "
          f"(packing, copies and cells included)\n")
    print("| kernel | launches | total ms | avg us | algorithmic GB | GB/s | frac of 8 TB/s | PMC GB (fetch x2 + write) |")
    print("|---|---|---|---|---|---|---|---|")
    tot_ms = tot_alg = 0.0
    other = []
    for row in trace:
        name = row["Name"]
        short = next((k for k in alg if k in name), None)
        if short is None:
            other.append(row)
            continue
        ms = float(row.get("TotalDurationNs") or float(row["AverageNs"]) * int(row["Calls"])) / 1e6
        fb = next((v for k, v in fetch.items() if short in k), float("nan")) * 1024 * 2
        wb = next((v for k, v in write.items() if short in k), float("nan")) * 1024
        gbs = alg[short] / (ms * 1e-3) / 1e9
        tot_ms += ms
        tot_alg += alg[short]
        rec["kernels"][short] = {"launches": int(row["Calls"]), "total_ms": ms, "algorithmic_bytes": alg[short],
                                 "pmc_fetch_bytes_x2": fb, "pmc_write_bytes": wb, "pmc_bytes": fb + wb}
        print(f"| {short} | {row['Calls']} | {ms:.3f} | {float(row['AverageNs']) / 1e3:.1f} | {alg[short] / 1e9:.2f} | "
              f"{gbs:.0f} | {gbs / HBM_PEAK_GBS:.3f} | {(fb + wb) / 1e9:.2f} |")
    keys = next((r for r in other if "preload_keys_kernel" in r["Name"]), None)
    if keys:
        kms = float(keys["AverageNs"]) * int(keys["Calls"]) / 1e6
        print(f"| preload_keys_kernel | {keys['Calls']} | {kms:.3f} | {float(keys['AverageNs']) / 1e3:.1f} | "
              f"(24 B per spectrum) | | | |")
    print(f"\nScan + write: {tot_alg / 1e9:.2f} GB in {tot_ms:.3f} ms = {tot_alg / tot_ms / 1e6:.0f} GB/s "
          f"({tot_alg / tot_ms / 1e6 / HBM_PEAK_GBS:.3f} of peak).")
    print("\nOther kernels in the same command (the DLA-sample generator at S = 10^4 and 10^5, 6 calls each "
          "incl. warm-up; the runtime's copies):\n")
    print("| kernel | calls | avg us | max us |")
    print("|---|---|---|---|")
    for r in other:
        if "preload_keys_kernel" in r["Name"]:
            continue
        print(f"| {r['Name'].replace('gpdla::(anonymous namespace)::', '').split('(')[0]} | {r['Calls']} | "
              f"{float(r['AverageNs']) / 1e3:.1f} | {float(r['MaxNs']) / 1e3:.1f} |")
    for k in ("dla_samples_S10000", "dla_samples_S100000"):
        print(f"\n{k}: {bench[k]['wall_ms']:.3f} ms wall per call ({bench[k]['note']})")
    if json_out:
        Path(json_out).write_text(json.dumps(rec, indent=1))


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2] if len(sys.argv) > 2 else None)
