#!/usr/bin/env python
"""The BERT text branch inside one profiled training step (dev tool): wall span, kernel count and
summed kernel time of the BERT forward and backward, and (--list) their kernels.

    python tools/text_branch.py gpurun_out/prof/run_results.db [--list]

Step = the last full im2col-to-im2col window (tools/step_phases.py).  Forward span: the step's
bert_embed_kernel up to the next im2col (the graph runs the text branch before Swin); backward span:
the first BERT-only kernel of the backward (grad_scale; the top layer's LayerNorm backward precedes
it) to the end of bert_embed_bwd, plus the kernels right after it on the same queue (the text
group's AdamW)."""
import argparse
import sqlite3

from rocprof_summary import short_name


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("db")
    ap.add_argument("--list", action="store_true")
    a = ap.parse_args()
    c = sqlite3.connect(a.db)
    rows = c.execute("select name, start, end, queue_id from kernels order by start").fetchall()
    opens = [i for i, r in enumerate(rows) if "im2col_kernel" in r[0]]
    a_i, b_i = opens[-2], opens[-1]
    t0 = rows[a_i][1]
    # forward: the embedding kernel issued before this step's im2col
    e_i = max(i for i in range(opens[-3] if len(opens) > 2 else 0, a_i) if "bert_embed_kernel" in rows[i][0])
    fwd = rows[e_i:a_i]
    # backward: first grad_scale after the decoder backward, back two (the top layer's LN backward +
    # its reduce), to bert_embed_bwd
    g_i = next(i for i in range(a_i, b_i) if "grad_scale" in rows[i][0])
    q = rows[g_i][3]
    j, back = g_i, 0
    while j > a_i and back < 2:
        j -= 1
        if rows[j][3] == q:
            back += 1
    e2 = next(i for i in range(g_i, b_i) if "bert_embed_bwd" in rows[i][0])
    bwd = [r for r in rows[j:e2 + 1] if r[3] == q]
    tail = [r for r in rows[e2 + 1:b_i] if r[3] == q][:3]
    print(f"step (im2col to im2col): {(rows[b_i][1] - t0) / 1e3:.1f} us")
    for tag, ks in (("fwd", fwd), ("bwd", bwd), ("bwd tail (same queue)", tail)):
        if not ks:
            continue
        wall = (max(r[2] for r in ks) - ks[0][1]) / 1e3
        busy = sum(r[2] - r[1] for r in ks) / 1e3
        print(f"bert {tag}: {len(ks)} kernels, wall {wall:.1f} us, kernel time {busy:.1f} us, "
              f"start {(ks[0][1] - t0) / 1e3:.1f} us after im2col")
        if a.list:
            for r in ks:
                print(f"   {(r[1] - t0) / 1e3:9.1f} {(r[2] - r[1]) / 1e3:7.1f} q{r[3]} {short_name(r[0])[:70]}")


if __name__ == "__main__":
    main()
