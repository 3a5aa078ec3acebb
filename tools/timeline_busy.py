#!/usr/bin/env python3
"""Busy fraction of the GPU over a rocprofv3 kernel trace (--kernel-trace --output-format csv): the
union of all kernel intervals over the span from the first third of the bench's chain kernels (past
the warm-up) to the last kernel, the idle gaps between them, and the per-kernel totals.

    python3 tools/timeline_busy.py <..._kernel_trace.csv>"""
import collections
import csv
import sys

CHAIN = ("weights_i8", "gemm_i8", "ldl_mfma", "prep_kernel", "convert", "reduce")


def main(path):
    rows = list(csv.DictReader(open(path)))
    ks = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"], r["Queue_Id"]) for r in rows)
    chain = [k for k in ks if any(t in k[2] for t in CHAIN)]
    t0, t1 = chain[len(chain) // 3][0], chain[-1][1]
    seg = [k for k in ks if k[0] >= t0 and k[1] <= t1]
    busy, gaps = 0, []
    cur_s, cur_e = seg[0][0], seg[0][1]
    for s, e, n, _ in seg[1:]:
        if s > cur_e:
            busy += cur_e - cur_s
            gaps.append((s - cur_e, n))
            cur_s, cur_e = s, e
        else:
            cur_e = max(cur_e, e)
    busy += cur_e - cur_s
    span = t1 - t0
    print(f"span {span / 1e6:.2f} ms, GPU busy {busy / 1e6:.2f} ms ({busy / span:.3f}); {len(gaps)} idle gaps, "
          f"{sum(g for g, _ in gaps) / 1e6:.3f} ms in all")
    for g, n in sorted(gaps, reverse=True)[:5]:
        print(f"  gap {g / 1e3:.1f} us before {n[:70]}")
    tot, cnt = collections.defaultdict(float), collections.Counter()
    for s, e, n, _ in seg:
        key = n.replace("gpdla::(anonymous namespace)::", "").replace("void ", "").split("(")[0]
        tot[key] += (e - s) / 1e6
        cnt[key] += 1
    for k in sorted(tot, key=lambda k: -tot[k]):
        print(f"{k[:48]:48s} {cnt[k]:6d} launches {tot[k]:9.2f} ms  avg {tot[k] / cnt[k] * 1e3:8.1f} us")
    print("queues:", dict(collections.Counter(k[3] for k in seg)))


if __name__ == "__main__":
    main(sys.argv[1])
