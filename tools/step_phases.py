#!/usr/bin/env python
"""Phase markers of the last full training step in a rocprofv3 kernel trace (dev tool): first / last
start of the BERT, Swin and decoder kernels of the forward and backward, the optimizer launches, and
the step's wall time, to see which branch is on the critical path.

    python tools/step_phases.py gpurun_out/prof/run_results.db
"""
import sqlite3
import sys

from rocprof_summary import short_name

MARK = {"bert fwd": ("mhaL_fwd", "bert_embed_kernel"), "bert bwd": ("mhaL_bwd", "bert_embed_bwd"),
        "swin fwd": ("wattn_qkv_fwd", "im2col"), "swin bwd": ("wattn_bwd",), "decoder fwd": ("dec_ca_fwd", "dec_step_fwd"),
        "decoder bwd": ("dec_ca_bwd", "dec_step_bwd"), "adamw": ("adamw",)}


def main():
    c = sqlite3.connect(sys.argv[1])
    rows = c.execute("select name, start, end, queue_id from kernels order by start").fetchall()
    opens = [i for i, r in enumerate(rows) if "im2col_kernel" in r[0]]
    a, b = opens[-2], opens[-1]
    seg = rows[a - 400:b]
    t0 = rows[a][1]
    print(f"step (im2col to im2col): {(rows[b][1] - t0) / 1e3:.1f} us")
    for k, pats in MARK.items():
        hit = [r for r in seg if any(p in r[0] for p in pats) and r[1] >= rows[a - 400][1]]
        if hit:
            qs = sorted(set(r[3] for r in hit))
            print(f"{k:12s} n={len(hit):4d} first {(hit[0][1] - t0) / 1e3:9.1f} last_end {(max(r[2] for r in hit) - t0) / 1e3:9.1f}"
                  f" queues {qs}")
    for r in seg:
        if "adamw" in r[0]:
            print(f"   adamw {(r[1] - t0) / 1e3:9.1f} {(r[2] - r[1]) / 1e3:7.1f} q{r[3]}")


if __name__ == "__main__":
    main()
