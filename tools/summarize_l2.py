"""Per-dispatch counter averages of configs[4]'s three chain kernels from tools/profile_l2.sh's passes, and
the derived limiter figures (Little's law on the L1 -> L2 read stream, VALU issue cycles).

    python tools/summarize_l2.py gpurun_out/l2_<tag> profiles/round6/<tag>_c5_chain_counters   (.json + .md)
"""
import csv
import glob
import json
import sys
from collections import defaultdict
from pathlib import Path

KERNELS = {"gemm_i8_bst_kernel": "Gram + u GEMM (gemm_i8_bst_kernel)",
           "weights_i8_kernel<true>": "weights (weights_i8_kernel<true>)",
           "ldl_mfma_kernel<13, float>": "LDL^T (ldl_mfma_kernel<13, float>)"}
CUS, SIMDS, XCDS = 256, 1024, 8
LINE = 128          # bytes per TCP -> TCC read request (TCC_READ_SECTORS / TCP_TCC_READ_REQ = 4 x 32 B, measured)


def load(d: Path) -> dict:
    per = defaultdict(lambda: defaultdict(list))     # kernel -> counter -> per-dispatch values (pass-local)
    for p in "abcd":
        for f in glob.glob(str(d / p / "*counter_collection.csv")):
            for row in csv.DictReader(open(f)):
                name = row["Kernel_Name"].replace("(anonymous namespace)::", "").replace("void ", "")
                key = next((k for k in KERNELS if k in name.split("(")[0]), None)
                if key is None:
                    continue
                per[key][(p, row["Counter_Name"])].append(float(row["Counter_Value"]))
    out = {}
    for k, cs in per.items():
        avg = {}
        for (p, n), v in cs.items():
            avg.setdefault(n, {})[p] = sum(v) / len(v)
        out[k] = {n: (sum(v.values()) / len(v)) for n, v in avg.items()}   # GRBM is in every pass: mean
        out[k]["dispatches_per_pass"] = max(len(v) for v in cs.values())
    return out


def derive(c: dict) -> dict:
    cyc = c["GRBM_GUI_ACTIVE"] / XCDS                     # kernel cycles (each XCD counts its own)
    d = {"kernel_cycles": cyc}
    req = c.get("TCP_TCC_READ_REQ_sum", 0.0)
    if req:
        lat = c["TCP_TCC_READ_REQ_LATENCY_sum"] / req
        rate = req / CUS / cyc                              # read requests per clock per CU
        d.update({"l2_read_bytes": req * LINE, "l2_read_latency_cycles": lat,
                  "l2_read_bytes_per_clk_per_cu": rate * LINE,
                  "lines_in_flight_per_cu": rate * lat,       # Little's law
                  "tcc_hit_rate": c["TCC_HIT_sum"] / (c["TCC_HIT_sum"] + c["TCC_MISS_sum"]),
                  "sectors_per_request": c["TCC_READ_SECTORS_sum"] / req,
                  "tcp_pending_stall_frac": c["TCP_PENDING_STALL_CYCLES_sum"] / CUS / cyc,
                  "ta_data_stalled_by_tc_frac": c["TA_DATA_STALLED_BY_TC_CYCLES_sum"] / CUS / cyc})
    valu = c.get("SQ_INSTS_VALU", 0.0)
    if valu:
        trans = c.get("SQ_INSTS_VALU_TRANS_F32", 0.0) + c.get("SQ_INSTS_VALU_TRANS_F64", 0.0)
        # a wave64 VALU instruction holds a SIMD 4 cycles (16 lanes per clock, f32 and f64 alike on gfx950);
        # transcendentals 4x that
        issue = (4 * valu + 12 * trans) / SIMDS
        d.update({"valu_per_dispatch": valu, "valu_issue_cycles_per_simd": issue, "valu_issue_frac": issue / cyc,
                  "valu_mix": {n.replace("SQ_INSTS_VALU_", ""): c[n] / valu for n in sorted(c)
                               if n.startswith("SQ_INSTS_VALU_")}})
    return d


if __name__ == "__main__":
    src, dst = Path(sys.argv[1]), Path(sys.argv[2])
    raw = load(src)
    res = {k: {"counters": raw[k], "derived": derive(raw[k])} for k in raw}
    dst.with_suffix(".json").write_text(json.dumps(res, indent=1))
    lines = [f"# configs[4] chain counters ({src.name}; one stream, per dispatch = one spectrum x 100,001 samples)", "",
             "| kernel | cycles | L2 read GB | L2 latency (cyc) | B/clk/CU | lines in flight / CU | L2 hit | TCP pending-stall | VALU issue frac |",
             "|---|---|---|---|---|---|---|---|---|"]
    for k, label in KERNELS.items():
        if k not in res:
            continue
        d = res[k]["derived"]
        lines.append(f"| {label} | {d['kernel_cycles']:.3g} | {d.get('l2_read_bytes', 0) / 1e9:.2f} | "
                     f"{d.get('l2_read_latency_cycles', 0):.0f} | {d.get('l2_read_bytes_per_clk_per_cu', 0):.1f} | "
                     f"{d.get('lines_in_flight_per_cu', 0):.1f} | {d.get('tcc_hit_rate', 0):.3f} | "
                     f"{d.get('tcp_pending_stall_frac', 0):.2f} | {d.get('valu_issue_frac', 0):.2f} |")
    dst.with_suffix(".md").write_text("\n".join(lines) + "\n")
    print("\n".join(lines))
