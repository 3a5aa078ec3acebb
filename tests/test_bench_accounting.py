"""CPU checks of bench.py's work and traffic accounting (DESIGN.md sections 8, 10):
the per-eval flop / byte / int8-op formulas at the BASELINE configs, and the lookup of the
committed PMC traffic for configs[1] (fused fp64) and configs[4] (int8 panel-GEMM)."""
import importlib.util
import json
from pathlib import Path

import numpy as np
import pytest

ROOT = Path(__file__).resolve().parents[1]


@pytest.fixture(scope="module")
def bench():
    spec = importlib.util.spec_from_file_location("bench_under_test", ROOT / "bench.py")
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


def test_flops_and_bytes_per_eval(bench):
    # ~3.79e5 flop and 160,072 B per eval at n = 800, k = 20 (fp64)
    assert bench.algorithmic_flops_per_eval(800, 20) == pytest.approx(379466.667, rel=1e-6)
    assert bench.effective_bytes_per_eval(800, 20) == 160072
    # k = 50 (configs[4]): ~2.17e6 flop
    assert bench.algorithmic_flops_per_eval(800, 50) == pytest.approx(2174666.667, rel=1e-6)


def test_i8_ops_per_eval(bench):
    # 10 digit pairs x n slots x (1275 Gram + 50 u entries) x 2 ops at k = 50
    assert bench.i8_ops_per_eval(800, 50) == 2 * 10 * 800 * 1325
    # 24-bit Gram contraction: 6 pairs per Gram entry, the u entries keep 10
    assert bench.i8_ops_per_eval(800, 50, 6) == 2 * 800 * (6 * 1275 + 10 * 50)


def test_i8_roofline_uses_the_gemm_launches(bench):
    st = {"contraction_ms": 20.0, "contraction_launches": 20, "likelihood_ms": 30.0, "likelihood_launches": 2}
    r = bench.i8_roofline(st, 800, 50, Q=10, S=99, steps=2, path="panel-GEMM-int8-24")
    ops = bench.i8_ops_per_eval(800, 50, 6)
    # 20 GEMM launches of 1 ms over 10 spectra x 100 evals x 2 steps
    assert r["avg_launch_ms"] == 1.0 and r["evals_per_launch"] == 100
    assert r["achieved"] == pytest.approx(ops * 100 / 1e-3 / 1e12)
    assert r["frac"] == pytest.approx(r["achieved"] / bench.I8_PEAK_TOPS)
    assert r["whole_batch"]["avg_ms"] == 15.0


def test_panel_roofline_streams_record(bench):
    """With two panel streams the roofline is the timed region's GEMM launches, with
    the kernel's one-stream launch (measured after the timed region) nested beside it; the batch
    figures stay the timed region's.  A record without launch timing passes through unchanged."""
    st2 = {"contraction_ms": 32.0, "contraction_launches": 20, "likelihood_ms": 28.0, "likelihood_launches": 2}
    st1 = {"contraction_ms": 2.0, "contraction_launches": 2, "likelihood_ms": 16.0, "likelihood_launches": 1}
    timed = bench.i8_roofline(st2, 800, 50, Q=10, S=99, steps=2, path="panel-GEMM-int8-24")
    alone = bench.i8_roofline(st1, 800, 50, Q=1, S=99, steps=2, path="panel-GEMM-int8-24")
    r = bench.panel_roofline_streams(timed, alone, 2)
    assert r["avg_launch_ms"] == 1.6 and r["frac"] == pytest.approx(timed["frac"])
    assert r["one_stream"]["avg_launch_ms"] == 1.0 and r["one_stream"]["frac"] == pytest.approx(alone["frac"])
    assert r["one_stream"]["frac"] > r["frac"]
    assert r["whole_batch"] == timed["whole_batch"]
    f64 = bench.f64_gemm_roofline({**st1, "contraction_launches": 0}, 800, 50, 1, 99, 2)
    assert bench.panel_roofline_streams(f64, alone) is f64


def test_no_field_reads_as_a_fraction_above_one(bench):
    """Honest units: the int8 frac says what it measures, the batch's algorithmic rate
    is named as such and set against the FP32 matrix peak, and no 'fp64-equivalent' figure remains."""
    st = {"contraction_ms": 0.54, "contraction_launches": 1, "likelihood_ms": 0.47, "likelihood_launches": 1}
    r = bench.i8_roofline(st, 800, 50, Q=1, S=100000, steps=1, path="panel-GEMM-int8-24")
    assert "digit" in r["frac_meaning"] and "6" in r["frac_meaning"]
    wb = r["whole_batch"]
    assert "fp64_equivalent_tflops" not in wb and wb["fp32_matrix_peak_tflops"] == 157.3
    assert wb["algorithmic_over_fp32_matrix_peak"] == pytest.approx(wb["algorithmic_tflops"] / 157.3)
    assert 0 < wb["digit_frac_of_i8_peak"] < 1 and 0 < r["frac"] < 1
    assert "fp64_equivalent" not in (ROOT / "bench.py").read_text()


def test_profiled_traffic_lookup(bench):
    """Every bench workload's roofline traffic comes from the committed summary bench.py names, summed
    over that path's roofline-kernel launches; other shapes claim no profiled number."""
    t, src = bench.profiled_traffic(1024, 10000, 20, "fused")
    rows = json.loads(bench.PROFILE_SUMMARY.read_text())["kernels"]
    want = [e["hbm_bytes_per_launch"] for e in rows if e["kernel"].startswith("void gpdla::likelihood_kernel<20")]
    assert t is not None and t > 0 and t == want[0] and bench.PROFILE_SUMMARY.name in src
    for path, (f, names) in bench.PROFILE_SUMMARY_C5.items():
        tp, srcp = bench.profiled_traffic(128, 100000, 50, path)
        if not f.exists():          # not profiled on the current tree: no number is claimed
            assert (tp, srcp) == (None, None)
            continue
        rows = json.loads(f.read_text())["kernels"]
        # exact names: per-batch kernels whose names contain the GEMM's (convert_gemm_i8_kernel) excluded
        assert tp == sum(e["hbm_bytes_per_launch"] for e in rows if e["kernel"] in names) and tp > 0
        assert f.name in srcp and "convert" not in srcp
    # other workloads / paths: no profiled number is claimed
    assert bench.profiled_traffic(128, 100000, 50, "fused") == (None, None)
    assert bench.profiled_traffic(64, 10000, 20, "fused") == (None, None)

def test_widened_cpu_baseline(bench):
    """The widened rows' CPU restatements (beside alternatives.dla_samples / .ingest) run on the host
    and report positive one-core rates with their samples named."""
    w = bench.widened_cpu_baseline()
    for key, unit in (("generate_dla_samples", "samples/s"), ("preload_qsos", "pixels/s"), ("objective", "spectra/s")):
        assert w[key]["value"] > 0 and w[key]["unit"] == unit and w[key]["cores"] == 1 and w[key]["kind"] == "port"
        assert w[key]["sample"]


def test_ingest_profile_summary(bench):
    """alternatives.ingest's roofline traffic comes from the committed PMC summary of the same workload;
    the PMC bytes of each kernel sit within 10% of its algorithmic bytes (no wasted re-reads)."""
    kp = json.loads(bench.INGEST_PROFILE.read_text())["kernels"]
    for k in ("preload_scan_kernel", "preload_write_kernel"):
        assert kp[k]["launches"] == 11 and kp[k]["total_ms"] > 0
        assert abs(kp[k]["pmc_bytes"] / kp[k]["algorithmic_bytes"] - 1) < 0.10


def test_objective_flops_accounting(bench):
    """The objective leg's algorithmic flops: per valid pixel 3k^2 + 12k, per spectrum k^3."""
    y = np.array([[1.0, np.nan, 2.0], [np.nan, np.nan, 3.0]])
    assert bench.objective_flops(y, 4) == 2 * (3 * 16 + 48) + 64 + 1 * (3 * 16 + 48) + 64
