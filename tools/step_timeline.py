#!/usr/bin/env python
"""Kernel timeline of the last full training step in a rocprofv3 kernel trace (dev tool): one line
per kernel (start offset from the step's im2col, duration, queue, name) plus how much of the step ran
two or more kernels at once — whether captured graph branches overlapped at all.

    python tools/step_timeline.py gpurun_out/prof/run_results.db > timeline.txt
"""
import sqlite3
import sys

from rocprof_summary import short_name


def main():
    c = sqlite3.connect(sys.argv[1])
    rows = c.execute("select name, start, end, queue_id from kernels order by start").fetchall()
    opens = [i for i, r in enumerate(rows) if "im2col_kernel" in r[0]]
    a, b = opens[-2], opens[-1]
    t0, t1 = rows[a][1], rows[b][1]
    seg = [r for r in rows if r[2] > t0 and r[1] < t1]
    # time covered by >= 1 and >= 2 kernels (sweep over start / end events)
    ev = sorted([(max(r[1], t0), 1) for r in seg] + [(min(r[2], t1), -1) for r in seg])
    depth, last, busy, multi = 0, t0, 0, 0
    for t, d in ev:
        if depth >= 1:
            busy += t - last
        if depth >= 2:
            multi += t - last
        depth += d
        last = t
    print(f"step {(t1 - t0) / 1e3:.1f} us, {len(seg)} kernels, busy {busy / 1e3:.1f} us, "
          f">= 2 kernels at once {multi / 1e3:.1f} us")
    for r in seg:
        print(f"{(r[1] - t0) / 1e3:9.1f} {(r[2] - r[1]) / 1e3:7.1f} q{r[3]} {short_name(r[0])[:60]}")


if __name__ == "__main__":
    main()
