"""Per-kernel VGPRs / AGPRs / scratch / LDS / occupancy of every HIP translation unit of libgpdla, from
the compiler's resource report (hipcc -Rpass-analysis=kernel-resource-usage, gfx950).

    python tools/kernel_resources.py [out.md]      (default: print)
"""
import re
import subprocess
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
from gp_dla_detection_amd.build import CSRC, SOURCES  # noqa: E402

FIELDS = ("VGPRs", "AGPRs", "ScratchSize [bytes/lane]", "Occupancy [waves/SIMD]", "LDS Size [bytes/block]",
          "VGPRs Spill")


def report(src: Path) -> list:
    r = subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-c",
                        "--cuda-device-only", "-Wno-unused-result", "-Rpass-analysis=kernel-resource-usage",
                        "-o", "/dev/null", str(src)], capture_output=True, text=True, cwd=CSRC)
    rows, cur = [], None
    for line in r.stderr.splitlines():
        m = re.search(r"remark: Function Name: (\S+)", line)
        if m:
            cur = {"kernel": m.group(1), "file": src.name}
            rows.append(cur)
            continue
        m = re.search(r"remark:\s+([^:]+): (\S+) \[", line)
        if m and cur is not None and m.group(1).strip() in FIELDS:
            cur[m.group(1).strip()] = m.group(2)
    return rows


def demangle(names):
    r = subprocess.run(["c++filt"], input="\n".join(names), capture_output=True, text=True)
    return r.stdout.splitlines() if r.returncode == 0 else names


if __name__ == "__main__":
    rows = [row for s in SOURCES if s.endswith(".hip") for row in report(CSRC / s)]
    names = demangle([r["kernel"] for r in rows])
    lines = ["| file | kernel | VGPRs | AGPRs | spilled VGPRs | scratch B/lane | waves/SIMD | LDS B/block |",
             "|---|---|---|---|---|---|---|---|"]
    for r, n in zip(rows, names):
        n = n.replace("gpdla::(anonymous namespace)::", "")
        lines.append(f"| {r['file']} | `{n}` | {r.get('VGPRs', '')} | {r.get('AGPRs', '')} | {r.get('VGPRs Spill', '')} | "
                     f"{r.get('ScratchSize [bytes/lane]', '')} | {r.get('Occupancy [waves/SIMD]', '')} | "
                     f"{r.get('LDS Size [bytes/block]', '')} |")
    text = "\n".join(lines) + "\n"
    if len(sys.argv) > 1:
        Path(sys.argv[1]).write_text("# Kernel resources (hipcc -Rpass-analysis=kernel-resource-usage, gfx950)\n\n" + text)
    print(text)
