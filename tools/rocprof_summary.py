#!/usr/bin/env python
"""Summarise a rocprofv3 (ROCm 7 rocpd SQLite) kernel trace as a per-kernel stats table.

    python tools/rocprof_summary.py gpurun_out/prof/run_results.db [--last N] [--top 40] > profiles/rX_stats.md

Columns match `rocprofv3 --stats` (calls, total / average / min / max duration in microseconds,
share of total kernel time).  --last N keeps only the dispatches of the last N training steps (the
timed graph replays of `bench.py --roofline-steps 0 --agent-steps 0`): everything after the optimizer
launch that precedes them, up to the last optimizer launch, so warm-up / capture / eager steps and
one-off work are excluded.  Steps are delimited by the patch-embedding im2col launch that opens
every forward (the optimizer now runs as several sub-range launches per step); the window is the
N steps before the last im2col.  Kernel names are shortened (template args kept)."""
import argparse
import re
import sqlite3
from collections import defaultdict


def short_name(name):
    mg = re.match(r"_ZN12_GLOBAL__N_1(\d+)", name)   # mangled (bf16 args defeat c++filt): keep the name
    if mg:
        ln = int(mg.group(1))
        name = name[mg.end():mg.end() + ln] + ("<...>" if name[mg.end() + ln:].startswith("I") else "")
    short = re.sub(r"\(anonymous namespace\)::", "", name)
    short = re.sub(r"\((?:[^()]|\([^()]*\))*\)$", "", short).replace("void ", "")
    return short if len(short) <= 90 else short[:87] + "..."


def load(path):
    c = sqlite3.connect(path)
    cols = [r[1] for r in c.execute("pragma table_info(kernels)").fetchall()]
    start = "start" if "start" in cols else ("start_ns" if "start_ns" in cols else None)
    if start is None:
        rows = c.execute("select name, duration from kernels").fetchall()
        return [(n, 0, d) for n, d in rows]
    return c.execute(f"select name, {start}, duration from kernels order by {start}").fetchall()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("db")
    ap.add_argument("--last", type=int, default=0)
    ap.add_argument("--top", type=int, default=40)
    a = ap.parse_args()
    rows = load(a.db)
    opens = [i for i, r in enumerate(rows) if "im2col_kernel" in r[0]]
    steps = len(opens) or 1
    window = "all dispatches"
    if a.last and len(opens) > a.last:
        rows = rows[opens[-a.last - 1]:opens[-1]]
        steps = a.last
        window = f"{a.last} training steps (from forward #{len(opens) - a.last} to the last forward's start)"
    agg = defaultdict(lambda: [0, 0.0, 0.0, float("inf"), 0.0])
    for name, _, d in rows:
        e = agg[name]
        e[0] += 1
        e[1] += d
        e[3] = min(e[3], d)
        e[4] = max(e[4], d)
    total = sum(e[1] for e in agg.values())
    print(f"# rocprofv3 --kernel-trace summary: {a.db}")
    print(f"# window: {window}")
    print(f"# total kernel time {total / 1e6:.3f} ms over {sum(e[0] for e in agg.values())} dispatches; "
          f"{steps} training steps -> {total / 1e6 / steps:.2f} ms of kernels per step\n")
    print("| kernel | calls | total_us | avg_us | min_us | max_us | pct | us/step |")
    print("|---|---|---|---|---|---|---|---|")
    for name, (n, s, _, lo, hi) in sorted(agg.items(), key=lambda kv: -kv[1][1])[:a.top]:
        print(f"| `{short_name(name)}` | {n} | {s / 1e3:.1f} | {s / n / 1e3:.2f} | {lo / 1e3:.2f} | {hi / 1e3:.2f} | "
              f"{100 * s / total:.2f} | {s / 1e3 / steps:.1f} |")


if __name__ == "__main__":
    main()
