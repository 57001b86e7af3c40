"""Step timeline from a rocprofv3 kernel trace (``--kernel-trace --output-format csv``): per stream / queue busy time,
the union of busy time (GPU idle = launch / dependency gaps), time with two or more streams busy (overlap), and the
kernels that run ALONE longest (the exposed critical path). The window is the last ``--steps`` steps, found by the
embedding forward kernel that starts every step.

    python tools/timeline.py <kernel_trace.csv> [--steps N] [--marker embed_fwd] [--top 25]"""
import argparse
import collections
import csv


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--marker", default="embed_fwd")
    ap.add_argument("--top", type=int, default=25)
    a = ap.parse_args()
    rows = list(csv.DictReader(open(a.trace)))
    qk = "Stream_Id" if "Stream_Id" in rows[0] else "Queue_Id"
    ks = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"], r[qk]) for r in rows]
    ks.sort()
    starts = [k[0] for k in ks if a.marker in k[2]]
    if len(starts) < a.steps + 1:
        raise SystemExit(f"found {len(starts)} '{a.marker}' markers")
    t0, t1 = starts[-a.steps - 1], starts[-1]
    win = [k for k in ks if k[0] >= t0 and k[0] < t1]
    wall = (t1 - t0) / a.steps
    per_q = collections.defaultdict(int)
    for s, e, n, q in win:
        per_q[q] += e - s
    # sweep: busy union, overlap, and time each kernel runs alone
    ev = []
    for i, (s, e, n, q) in enumerate(win):
        ev.append((s, 1, i))
        ev.append((e, -1, i))
    ev.sort()
    active = set()
    last = t0
    busy = over = 0
    alone = collections.defaultdict(int)
    gaps = collections.defaultdict(lambda: [0, 0])
    prev_end = None
    for t, d, i in ev:
        dt = t - last
        if dt > 0 and not active and prev_end is not None:
            g = gaps[(prev_end.split("(")[0][-45:], win[i][2].split("(")[0][-45:])]
            g[0] += dt
            g[1] += 1
        if d < 0:
            prev_end = win[i][2]
        if dt > 0 and active:
            busy += dt
            qs = {win[j][3] for j in active}
            if len(qs) > 1:
                over += dt
            if len(active) == 1:
                alone[win[next(iter(active))][2]] += dt
        last = t
        if d > 0:
            active.add(i)
        else:
            active.discard(i)
    print(f"wall/step {wall / 1e3:.1f} us  busy {busy / a.steps / 1e3:.1f} us  idle {(t1 - t0 - busy) / a.steps / 1e3:.1f} us"
          f"  multi-stream overlap {over / a.steps / 1e3:.1f} us")
    for q, v in sorted(per_q.items(), key=lambda x: -x[1]):
        print(f"  stream/queue {q}: {v / a.steps / 1e3:.1f} us busy/step")
    tot = collections.Counter()
    for n, v in alone.items():
        tot[n.split("(")[0][-90:]] += v
    print("idle gaps by (kernel before -> kernel after): us/step, gaps/step")
    for (x, y), (v, c) in sorted(gaps.items(), key=lambda kv: -kv[1][0])[:a.top]:
        print(f"  {v / a.steps / 1e3:8.1f} {c / a.steps:6.1f}  {x} -> {y}")
    print("kernels running alone (us/step):")
    for n, v in tot.most_common(a.top):
        print(f"  {v / a.steps / 1e3:8.1f}  {n}")


if __name__ == "__main__":
    main()
