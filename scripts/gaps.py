"""GPU idle gaps of the last timed step in a rocprofv3 kernel trace.

    python scripts/gaps.py gpurun_out/run/prof8/p_kernel_trace.csv [first_kernel] [last_kernel]

The step is the span from the last launch of ``first_kernel`` (default binize: the fit's first kernel) to
the following launch of ``last_kernel`` (default predict_heap: the transform).  Prints the span, the idle time
between kernels (the host-bound part), the largest gaps and the per-kernel busy time.
"""
import collections
import csv
import sys


def main():
    path = sys.argv[1]
    first = sys.argv[2] if len(sys.argv) > 2 else "binize"
    last = sys.argv[3] if len(sys.argv) > 3 else "predict_heap"
    rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))
    s = [i for i, r in enumerate(rows) if first in r["Kernel_Name"]][-1]
    e = next(i for i in range(s, len(rows)) if last in rows[i]["Kernel_Name"])
    seg = rows[s:e + 1]
    t0, t1 = int(seg[0]["Start_Timestamp"]), int(seg[-1]["End_Timestamp"])
    gaps, busy, end = [], collections.Counter(), t0
    for r in seg:
        a, b = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        if a > end:
            gaps.append((a - end, r["Kernel_Name"][:70]))
        busy[r["Kernel_Name"][:60]] += b - a
        end = max(end, b)
    print(f"step span {(t1 - t0) / 1e6:.2f} ms, idle {sum(g for g, _ in gaps) / 1e6:.2f} ms in {len(gaps)} gaps, "
          f"{len(seg)} kernels")
    for g, n in sorted(gaps, reverse=True)[:12]:
        print(f"  {g / 1e3:8.1f} us before {n}")
    for k, v in busy.most_common(14):
        print(f"{v / 1e6:8.2f} ms {k}")


if __name__ == "__main__":
    main()
