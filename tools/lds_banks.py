#!/usr/bin/env python3
"""LDS bank-conflict model of the split-bf16 GEMM staging images (csrc/kernels/gemm.hip, gemm_x6s_kernel).

Image row r = 208 B: [hi k0..31 | mid | lo | pad]; 16-B k-chunks optionally XOR-swizzled by (r ^ r>>3) & 3.
Reads: ds_read_b128, lane l -> row l&31, chunk 2*ks + (l>>5); writes: ds_write_b64 of a thread's 4 k at
row 4g+i, with (g, c) = (t>>3, t&7) for k-contiguous sources and (t&31, t>>5) for mn-contiguous ones.
Lane groups and bank widths from MI355X_MICROARCH.md (LDS table).  Prints the worst N-way per case.
"""
P = 52  # dwords per row


def swz(r):
    return (r ^ (r >> 3)) & 3


def read_ways(use_swz):
    g0 = list(range(0, 4)) + list(range(12, 16)) + list(range(20, 28))
    g1 = list(range(4, 12)) + list(range(16, 20)) + list(range(28, 32))
    worst = 0
    for grp in (g0, g1, [32 + x for x in g0], [32 + x for x in g1]):
        for p in range(3):
            for ks in range(2):
                banks = {}
                for lane in grp:
                    r, h = lane & 31, lane >> 5
                    kc = 2 * ks + h
                    d = r * P + 16 * p + 4 * (kc ^ swz(r) if use_swz else kc)
                    for b in range(4):
                        banks.setdefault((d + b) % 64, set()).add(d + b)
                worst = max(worst, max(len(v) for v in banks.values()))
    return worst


def write_ways(kcontig, use_swz):
    worst = 0
    for i in range(4):
        for p in range(3):
            for g0 in range(0, 64, 16):
                banks = {}
                for lane in range(g0, g0 + 16):
                    g, c = (lane // 8, lane % 8) if kcontig else (lane % 32, lane // 32)
                    r = 4 * g + i
                    cc = 2 * ((c >> 1) ^ swz(r)) + (c & 1) if use_swz else c
                    d = r * P + 16 * p + 2 * cc
                    for b in range(2):
                        banks.setdefault((d + b) % 32, set()).add(d + b)
                worst = max(worst, max(len(v) for v in banks.values()))
    return worst


if __name__ == "__main__":
    print("k-contiguous source, no swizzle : read %d-way, write %d-way" % (read_ways(False), write_ways(True, False)))
    print("mn-contiguous source, no swizzle: read %d-way, write %d-way" % (read_ways(False), write_ways(False, False)))
    print("mn-contiguous source, swizzled  : read %d-way, write %d-way" % (read_ways(True), write_ways(False, True)))
