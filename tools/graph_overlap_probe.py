#!/usr/bin/env python
"""Does the HIP graph executor run independent captured branches concurrently? (dev probe, GPU box)

Chain A: many small dependent kernels (a latency-bound chain, like the BERT text branch) on a side
stream; chain B: a few chip-filling matmuls (like the Swin backbone) on the capturing stream; both
forked from and joined into the capture stream.  Replay times of A alone, B alone and A || B: if the
executor overlaps branches, A || B ~ max(A, B); if it serialises them, ~ A + B.  Also the same with
the side chain captured FIRST vs SECOND (capture order).

    python tools/graph_overlap_probe.py
"""
import time

import torch


def timed(g, n=20):
    for _ in range(3):
        g.replay()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(n):
        g.replay()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / n * 1e3


def main():
    dev = torch.device("cuda")
    side = torch.cuda.Stream()
    small = torch.randn(320, 768, device=dev)
    sw = torch.randn(768, 768, device=dev, dtype=torch.float16)
    sx = small.half()
    big_a = torch.randn(8192, 4096, device=dev, dtype=torch.bfloat16)
    big_b = torch.randn(4096, 4096, device=dev, dtype=torch.bfloat16)

    def chain_a():
        y = sx
        for _ in range(150):
            y = torch.nn.functional.gelu(y @ sw)
        return y

    def chain_b():
        y = None
        for _ in range(12):
            y = big_a @ big_b
        return y

    def capture(body):
        g = torch.cuda.CUDAGraph()
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):
            body()
        torch.cuda.current_stream().wait_stream(s)
        torch.cuda.synchronize()
        with torch.cuda.graph(g):
            body()
        torch.cuda.synchronize()
        return g

    def both(side_first):
        def body():
            main = torch.cuda.current_stream()
            side.wait_stream(main)
            if side_first:
                with torch.cuda.stream(side):
                    chain_a()
                chain_b()
            else:
                chain_b()
                with torch.cuda.stream(side):
                    chain_a()
            main.wait_stream(side)
        return body

    def interleaved():
        """A's 150 steps and B's 12 issued alternately (A on the side stream): same graph edges as
        both(), different node creation order"""
        main = torch.cuda.current_stream()
        side.wait_stream(main)
        ya, yb = sx, None
        for i in range(150):
            with torch.cuda.stream(side):
                ya = torch.nn.functional.gelu(ya @ sw)
            if i % 12 == 0 and i < 144:
                yb = big_a @ big_b
        main.wait_stream(side)
        return ya, yb

    ti = timed(capture(interleaved))
    ta = timed(capture(chain_a))
    tb = timed(capture(chain_b))
    t1 = timed(capture(both(True)))
    t2 = timed(capture(both(False)))
    print(f"A alone {ta:.3f} ms, B alone {tb:.3f} ms, A+B {ta + tb:.3f}, max {max(ta, tb):.3f}")
    print(f"A || B, side chain captured first: {t1:.3f} ms; captured second: {t2:.3f} ms; interleaved: {ti:.3f} ms")
    # two latency-bound chains (neither fills the chip): concurrent branches would take ~max
    sx2 = sx.clone()

    def chain_c():
        y = sx2
        for _ in range(150):
            y = torch.nn.functional.gelu(y @ sw)
        return y

    def two_small():
        main = torch.cuda.current_stream()
        side.wait_stream(main)
        with torch.cuda.stream(side):
            chain_a()
        chain_c()
        main.wait_stream(side)
    tc = timed(capture(chain_c))
    t3 = timed(capture(two_small))
    print(f"two latency-bound chains: alone {ta:.3f} / {tc:.3f} ms, sum {ta + tc:.3f}, captured on two streams {t3:.3f} ms")
    # the same two chains as two graphs replayed on two streams
    ga, gc = capture(chain_a), capture(chain_c)
    s2 = torch.cuda.Stream()
    for _ in range(3):
        ga.replay()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(20):
        s2.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s2):
            ga.replay()
        gc.replay()
        torch.cuda.current_stream().wait_stream(s2)
    torch.cuda.synchronize()
    print(f"  as two graphs replayed on two streams: {(time.perf_counter() - t0) / 20 * 1e3:.3f} ms")


if __name__ == "__main__":
    main()
