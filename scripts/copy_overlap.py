"""H2D copy / kernel overlap from a rocprofv3 run with --kernel-trace --memory-copy-trace (csv output).

    python scripts/copy_overlap.py <dir with *_kernel_trace.csv and *_memory_copy_trace.csv>

Prints the host-to-device copies (count, bytes when the trace has them, busy time), how much of the copy time ran
while at least one kernel was executing, and a coarse timeline (per 1 % of the span: copy-busy and kernel-busy
fractions) -- the evidence that a streamed (out-of-core) fit overlaps its PCIe traffic with compute."""
import csv
import glob
import os
import sys


def _rows(d, suffix):
    f = sorted(glob.glob(os.path.join(d, "**", f"*{suffix}"), recursive=True))
    if not f:
        sys.exit(f"no *{suffix} under {d}")
    return list(csv.DictReader(open(f[0])))


def _union(iv):
    out = []
    for s, e in sorted(iv):
        if out and s <= out[-1][1]:
            out[-1][1] = max(out[-1][1], e)
        else:
            out.append([s, e])
    return out


def _overlap(a, b):
    """total length of the intersection of two sorted disjoint interval lists"""
    i = j = 0
    tot = 0
    while i < len(a) and j < len(b):
        s, e = max(a[i][0], b[j][0]), min(a[i][1], b[j][1])
        if e > s:
            tot += e - s
        if a[i][1] < b[j][1]:
            i += 1
        else:
            j += 1
    return tot


def main(d):
    kr = _rows(d, "kernel_trace.csv")
    cr = _rows(d, "memory_copy_trace.csv")
    kern = _union((int(r["Start_Timestamp"]), int(r["End_Timestamp"])) for r in kr)
    dcol = next((c for c in cr[0] if "Direction" in c), None) if cr else None
    h2d = [r for r in cr if dcol is None or "HOST_TO_DEVICE" in r[dcol].upper() or "H2D" in r[dcol].upper()]
    bcol = next((c for c in (cr[0] if cr else {}) if "Bytes" in c or c == "Size"), None)
    civ = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"])) for r in h2d]
    cu = _union(civ)
    cbusy = sum(e - s for s, e in cu)
    ov = _overlap(cu, kern)
    nbytes = sum(int(float(r[bcol])) for r in h2d) if bcol else None
    t0 = min([s for s, _ in kern] + [s for s, _ in cu])
    t1 = max([e for _, e in kern] + [e for _, e in cu])
    print(f"span {(t1 - t0) / 1e9:.3f} s; kernels busy {sum(e - s for s, e in kern) / 1e9:.3f} s in {len(kr)} launches")
    print(f"H2D copies: {len(h2d)}" + (f", {nbytes / 1e9:.1f} GB" if nbytes else "") +
          f", busy {cbusy / 1e9:.3f} s" + (f" ({nbytes / cbusy:.1f} GB/s while copying)" if nbytes else ""))
    print(f"H2D busy time with a kernel running: {ov / 1e9:.3f} s = {100.0 * ov / max(cbusy, 1):.1f} % of the copy time")
    if cu:
        # inside the streaming window (first copy start .. last copy end): how much of the kernel work ran while a
        # copy was in flight (the per-chunk compute hidden under the PCIe stream)
        win = [[cu[0][0], cu[-1][1]]]
        kin = [[max(s, win[0][0]), min(e, win[0][1])] for s, e in kern if e > win[0][0] and s < win[0][1]]
        kb = sum(e - s for s, e in kin)
        print(f"streaming window {(win[0][1] - win[0][0]) / 1e9:.3f} s: copies busy {100.0 * cbusy / (win[0][1] - win[0][0]):.1f} %, "
              f"kernels busy {kb / 1e9:.3f} s, of which {100.0 * _overlap(kin, cu) / max(kb, 1):.1f} % under a running copy")
        after = sum(e - s for s, e in kern if s >= win[0][1])
        print(f"after the stream: kernels busy {after / 1e9:.3f} s (the tree levels: they need every row's bins)")
    nb = 100
    w = (t1 - t0) / nb
    print("timeline (1 % bins): copy-busy % / kernel-busy %")
    line = []
    for b in range(nb):
        s, e = t0 + b * w, t0 + (b + 1) * w
        cb = _overlap(cu, [[s, e]]) / w * 100
        kb = _overlap(kern, [[s, e]]) / w * 100
        line.append(f"{cb:3.0f}/{kb:3.0f}")
        if len(line) == 10:
            print("  " + "  ".join(line))
            line = []


if __name__ == "__main__":
    main(sys.argv[1])
