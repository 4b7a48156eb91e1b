"""Print the first kernels of the last timed step of a rocprofv3 kernel trace (from the end of the previous
step's predict), with start offsets, gaps and streams: the fit prologue before the binning."""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
k = int(sys.argv[2]) if len(sys.argv) > 2 else 30
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
idx = [i for i, r in enumerate(rows) if "predict_heap" in r["Kernel_Name"]]
a, b = idx[-2], idx[-1]
t0 = prev = int(rows[a]["End_Timestamp"])
for r in rows[a + 1:b + 1][:k]:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    print(f"{(s - t0) / 1e3:9.1f} +{(s - prev) / 1e3:8.1f} dur {(e - s) / 1e3:8.1f} s{r['Stream_Id']} "
          f"{r['Kernel_Name'][:80]}")
    prev = max(prev, e)
