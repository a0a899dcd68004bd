#!/usr/bin/env python
"""Idle time of the GPU inside the timed training steps of a rocprofv3 kernel trace (dev tool).

    python tools/timeline_gaps.py gpurun_out/prof/run_results.db [--last 5]

Per step (delimited by the patch-embedding im2col launch that opens every forward): wall time, the union of
busy intervals over all queues, idle = wall - union, and the largest idle gaps with the kernels on
either side (the launch-latency-bound stretches of the step)."""
import argparse
import sqlite3

from rocprof_summary import short_name


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("db")
    ap.add_argument("--last", type=int, default=5)
    ap.add_argument("--top", type=int, default=15)
    a = ap.parse_args()
    c = sqlite3.connect(a.db)
    rows = c.execute("select name, start, end, queue_id from kernels order by start").fetchall()
    opens = [i for i, r in enumerate(rows) if "im2col_kernel" in r[0]]
    ends = [i - 1 for i in opens][-(a.last + 1):]
    tot_idle, tot_wall = 0.0, 0.0
    gaps = []
    for s in range(len(ends) - 1):
        seg = rows[ends[s] + 1:ends[s + 1] + 1]
        t0, t1 = seg[0][1], max(r[2] for r in seg)
        busy, cur_s, cur_e = 0, None, None
        last = None
        for name, st, en, q in seg:
            if cur_e is None or st > cur_e:
                if cur_e is not None:
                    busy += cur_e - cur_s
                    gaps.append((st - cur_e, short_name(last), short_name(name)))
                cur_s, cur_e = st, en
            else:
                cur_e = max(cur_e, en)
            if en >= cur_e:
                last = name
        busy += cur_e - cur_s
        wall = t1 - t0
        tot_idle += wall - busy
        tot_wall += wall
        print(f"step {s}: wall {wall / 1e6:.2f} ms  busy {busy / 1e6:.2f} ms  idle {(wall - busy) / 1e6:.2f} ms  "
              f"kernels {len(seg)}")
    n = max(1, len(ends) - 1)
    print(f"mean: wall {tot_wall / n / 1e6:.2f} ms, idle {tot_idle / n / 1e6:.2f} ms")
    agg = {}
    for g, p, q in gaps:
        k = (p, q)
        e = agg.setdefault(k, [0, 0.0])
        e[0] += 1
        e[1] += g
    print("\nidle by (kernel before, kernel after), us per step:")
    for (p, q), (cnt, g) in sorted(agg.items(), key=lambda kv: -kv[1][1])[:a.top]:
        print(f"  {g / 1e3 / n:8.1f} us  {cnt / n:6.1f}x  {p}  ->  {q}")


if __name__ == "__main__":
    main()
