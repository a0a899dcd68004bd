#!/usr/bin/env python
"""Summarise a rocprofv3 (ROCm 7 rocpd SQLite) kernel trace as a per-kernel stats table.

    python tools/rocprof_summary.py gpurun_out/prof/run_results.db > profiles/r1_xxx_stats.md

Columns match `rocprofv3 --stats` (calls, total / average / min / max duration in microseconds,
share of total kernel time).  Kernel names are shortened (template args kept)."""
import re
import sqlite3
import sys


def main(path, top=40):
    c = sqlite3.connect(path)
    rows = c.execute("select name, count(*), sum(duration), avg(duration), min(duration), max(duration) "
                     "from kernels group by name order by sum(duration) desc").fetchall()
    total = sum(r[2] for r in rows)
    steps = sum(r[1] for r in rows if "adamw_kernel" in r[0]) or 1   # one optimizer launch per training step
    print(f"# rocprofv3 --kernel-trace --stats summary: {path}")
    print(f"# total kernel time {total / 1e6:.3f} ms over {sum(r[1] for r in rows)} dispatches; "
          f"{steps} training steps (adamw launches) -> {total / 1e6 / steps:.2f} ms of kernels per step\n")
    print("| kernel | calls | total_us | avg_us | min_us | max_us | pct | us/step |")
    print("|---|---|---|---|---|---|---|---|")
    for name, n, s, a, lo, hi in rows[:top]:
        mg = re.match(r"_ZN12_GLOBAL__N_1(\d+)", name)   # mangled (bf16 args defeat c++filt): keep the name
        if mg:
            ln = int(mg.group(1))
            name = name[mg.end():mg.end() + ln] + ("<...>" if name[mg.end() + ln:].startswith("I") else "")
        short = re.sub(r"\(anonymous namespace\)::", "", name)
        short = re.sub(r"\((?:[^()]|\([^()]*\))*\)$", "", short).replace("void ", "")
        short = short if len(short) <= 90 else short[:87] + "..."
        print(f"| `{short}` | {n} | {s / 1e3:.1f} | {a / 1e3:.2f} | {lo / 1e3:.2f} | {hi / 1e3:.2f} | {100 * s / total:.2f} | {s / 1e3 / steps:.1f} |")


if __name__ == "__main__":
    main(sys.argv[1], int(sys.argv[2]) if len(sys.argv) > 2 else 40)
