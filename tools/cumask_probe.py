#!/usr/bin/env python
"""Can a latency-bound chain overlap a chip-filling one when each runs on a CU-masked stream? (dev
probe, GPU box)

graph_overlap_probe.py showed that a chain of small dependent kernels beside chip-filling GEMMs gains
nothing from running on a parallel branch (the big grids leave it no CUs).  Here the two chains run on
streams created with hipExtStreamCreateWithCUMask: chain A (150 small fp16 matmuls, like BERT's
launches) on a stream owning `--a-cus` CUs, chain B (bf16 4096-wide matmuls, like the Swin GEMMs) on
a stream owning the others.  Eager and as two HIP graphs replayed on the two masked streams (does a
graph replay keep the launch stream's CU mask?).

    python tools/cumask_probe.py [--a-cus 32]
"""
import argparse
import ctypes
import time

import torch


def masked_stream(lib, bits, ncu):
    words = (ncu + 31) // 32
    mask = (ctypes.c_uint32 * words)()
    for b in bits:
        mask[b // 32] |= 1 << (b % 32)
    h = ctypes.c_void_p()
    rc = lib.hipExtStreamCreateWithCUMask(ctypes.byref(h), ctypes.c_uint32(words), mask)
    if rc != 0:
        raise RuntimeError(f"hipExtStreamCreateWithCUMask: {rc}")
    return torch.cuda.ExternalStream(h.value)


def wall(fn, n=10):
    fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(n):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / n * 1e3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--a-cus", type=int, default=32)
    a = ap.parse_args()
    dev = torch.device("cuda")
    ncu = torch.cuda.get_device_properties(dev).multi_processor_count
    lib = ctypes.CDLL("libamdhip64.so")
    lib.hipExtStreamCreateWithCUMask.argtypes = [ctypes.POINTER(ctypes.c_void_p), ctypes.c_uint32,
                                                 ctypes.POINTER(ctypes.c_uint32)]
    sx = torch.randn(320, 768, device=dev).half()
    sw = torch.randn(768, 768, device=dev, dtype=torch.float16) / 28
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

    full_a, full_b = torch.cuda.Stream(), torch.cuda.Stream()
    # two CU splits: the first a_cus CU ids, or every (ncu / a_cus)-th id (spread over XCDs / SEs)
    step = max(1, ncu // a.a_cus)
    splits = {"low ids": set(range(a.a_cus)), "strided": set(range(0, ncu, step)[:a.a_cus])}
    print(f"{ncu} CUs; chain A = 150 x (320x768 @ 768x768 fp16 + gelu), chain B = 12 x 8192x4096x4096 bf16")

    def on(s, fn):
        with torch.cuda.stream(s):
            fn()

    def both(sa, sb):
        def f():
            cur = torch.cuda.current_stream()
            sa.wait_stream(cur)
            sb.wait_stream(cur)
            on(sa, chain_a)
            on(sb, chain_b)
            cur.wait_stream(sa)
            cur.wait_stream(sb)
        return f

    ta = wall(lambda: on(full_a, chain_a))
    tb = wall(lambda: on(full_b, chain_b))
    tab = wall(both(full_a, full_b))
    print(f"unmasked: A {ta:.3f} ms, B {tb:.3f} ms, A+B {ta + tb:.3f}, A || B {tab:.3f}")
    for name, bits in splits.items():
        sa = masked_stream(lib, sorted(bits), ncu)
        sb = masked_stream(lib, sorted(set(range(ncu)) - bits), ncu)
        ma = wall(lambda: on(sa, chain_a))
        mb = wall(lambda: on(sb, chain_b))
        mab = wall(both(sa, sb))
        print(f"masked ({name}, A {len(bits)} CUs / B {ncu - len(bits)}): A {ma:.3f} ms, B {mb:.3f} ms, "
              f"A || B {mab:.3f}")
        # graphs captured on ordinary streams, replayed on the masked ones
        graphs = []
        for body in (chain_a, chain_b):
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
            graphs.append(g)
        ga, gb = graphs

        def replay(g, s):
            return lambda: on(s, g.replay)

        def replay_both():
            cur = torch.cuda.current_stream()
            sa.wait_stream(cur)
            sb.wait_stream(cur)
            on(sa, ga.replay)
            on(sb, gb.replay)
            cur.wait_stream(sa)
            cur.wait_stream(sb)
        print(f"  graphs replayed: A on its masked stream {wall(replay(ga, sa)):.3f} ms (unmasked "
              f"{wall(replay(ga, full_a)):.3f}), B {wall(replay(gb, sb)):.3f} ms (unmasked {wall(replay(gb, full_b)):.3f}), "
              f"A || B {wall(replay_both):.3f} ms", flush=True)


if __name__ == "__main__":
    main()
