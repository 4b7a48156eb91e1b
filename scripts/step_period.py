"""Per-step GPU period (predict start to predict start) and busy time (union of kernel intervals) in a
rocprofv3 kernel trace of bench.py: period - busy is the time the GPU waited on the host."""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
iv = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]) for r in rows)
ps = [s for s, e, n in iv if "predict_heap" in n]
for a, b in zip(ps, ps[1:]):
    busy, cur_s, cur_e = 0, None, None
    for s, e, n in iv:
        if s < a or s >= b:
            continue
        e = min(e, b)
        if cur_e is None or s > cur_e:
            if cur_e is not None:
                busy += cur_e - cur_s
            cur_s, cur_e = s, e
        else:
            cur_e = max(cur_e, e)
    if cur_e is not None:
        busy += cur_e - cur_s
    print(f"period {(b - a) / 1e6:8.3f} ms  busy {busy / 1e6:8.3f} ms  idle {(b - a - busy) / 1e6:7.3f} ms")
