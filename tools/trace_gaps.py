"""Busy vs idle time of the GPU over the last N steps of a rocprofv3 kernel trace (kernel_trace.csv): the union of
kernel intervals, the gaps between them, and kernel counts.  python tools/trace_gaps.py <trace dir> [...]"""
import csv
import glob
import sys


def load(d):
    f = glob.glob(d + "/**/*kernel_trace.csv", recursive=True)[0]
    rows = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]) for r in csv.DictReader(open(f))]
    rows.sort()
    return rows


for d in sys.argv[1:]:
    rows = load(d)
    # the timed steps are the last part of the trace: take the last 60 % of kernels
    rows = rows[int(len(rows) * 0.4):]
    t0, t1 = rows[0][0], max(e for _, e, _ in rows)
    busy, cur_s, cur_e = 0, rows[0][0], rows[0][1]
    gaps = []
    for s, e, _ in rows[1:]:
        if s > cur_e:
            busy += cur_e - cur_s
            gaps.append(s - cur_e)
            cur_s, cur_e = s, e
        else:
            cur_e = max(cur_e, e)
    busy += cur_e - cur_s
    span = t1 - t0
    ksum = sum(e - s for s, e, _ in rows)
    gaps.sort()
    print(f"{d}: kernels {len(rows)} span {span/1e6:.2f} ms busy(union) {busy/1e6:.2f} ms ({100*busy/span:.1f} %) "
          f"sum(kernel) {ksum/1e6:.2f} ms gaps {len(gaps)} total {sum(gaps)/1e6:.2f} ms median {gaps[len(gaps)//2]/1e3 if gaps else 0:.1f} us "
          f"p90 {gaps[int(len(gaps)*0.9)]/1e3 if gaps else 0:.1f} us")
