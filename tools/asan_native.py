"""Exercise the host runtime (C++ batcher + libhdf5 shard IO/prefetcher) under ASan/UBSan.

SURVEY §5.2 asks for a sanitizer build of the native host code.  This script
loads the sanitized modules built by ``hetseq_amd.csrc.build.build_sanitized``
(same import names, separate directory) and drives every entry point with
randomised inputs, checking results against pure-Python/NumPy oracles.  It
must run with libasan preloaded (the Python interpreter is not instrumented):

    LD_PRELOAD=$(gcc -print-file-name=libasan.so):$(gcc -print-file-name=libstdc++.so) \\
    ASAN_OPTIONS=detect_leaks=0 python tools/asan_native.py build/native/asan

``tests/test_sanitizers.py`` does exactly that.  No torch import here: the
interpreter stays small and uninstrumented third-party code stays out of the
report.  Host code only (GPU sanitizers are not used on this platform).
"""
import importlib.machinery
import importlib.util
import os
import sys
import tempfile

import numpy as np


def load(name, d):
    path = [os.path.join(d, f) for f in os.listdir(d) if f.startswith(name + ".") and f.endswith(".so")]
    assert path, "no sanitized %s in %s" % (name, d)
    loader = importlib.machinery.ExtensionFileLoader(name, path[0])
    spec = importlib.util.spec_from_file_location(name, path[0], loader=loader)
    mod = importlib.util.module_from_spec(spec)
    loader.exec_module(mod)
    return mod


def oracle_batches(indices, lens, max_tokens, max_sentences, mult):
    """The reference's greedy cut rule, written out in Python."""
    out, batch, blens, slen = [], [], [], 0
    for k, idx in enumerate(indices):
        blens.append(lens[k])
        slen = max(slen, lens[k])
        if batch and (len(batch) == max_sentences or (len(batch) + 1) * slen > max_tokens):
            m = max(mult * (len(batch) // mult), len(batch) % mult)
            out.append(batch[:m])
            batch, blens = batch[m:], blens[m:]
            slen = max(blens)
        batch.append(idx)
    if batch:
        out.append(batch)
    return out


def check_batcher(nat, rng):
    for trial in range(300):
        n = int(rng.integers(0, 200))
        idx = rng.permutation(n).astype(np.int64)
        lens = rng.integers(1, 64, size=n).astype(np.int64)
        mt = int(rng.integers(64, 2000))
        ms = int(rng.integers(1, 40))
        mult = int(rng.integers(1, 9))
        got = [b.tolist() for b in nat.batch_by_size(idx, lens, mt, ms, mult)]
        assert got == oracle_batches(idx.tolist(), lens.tolist(), mt, ms, mult), trial
        c = int(rng.integers(1, 64))
        got = [b.tolist() for b in nat.batch_by_size(idx, c, mt, ms, mult)]
        assert got == oracle_batches(idx.tolist(), [c] * n, mt, ms, mult), trial
    for bad in (dict(bsz_mult=0), dict(max_sentences=0)):
        kw = dict(indices=np.arange(4), num_tokens=1, max_tokens=8, max_sentences=2, bsz_mult=1)
        kw.update(bad)
        try:
            nat.batch_by_size(**kw)
            raise AssertionError("invalid argument accepted")
        except ValueError:
            pass
    try:  # oversize sample
        nat.batch_by_size(np.arange(3), np.array([1, 99, 1]), 10, 4, 1)
        raise AssertionError("oversize sample accepted")
    except RuntimeError:
        pass


def make_shard(h5, path, n, S, P, rng, gzip=0):
    ids = rng.integers(0, 30000, size=(n, S)).astype(np.int32)
    mask = (rng.random((n, S)) < 0.9).astype(np.int8)
    seg = rng.integers(0, 2, size=(n, S)).astype(np.int8)
    pos = np.zeros((n, P), np.int32)
    mids = np.zeros((n, P), np.int32)
    for r in range(n):
        k = int(rng.integers(0, P + 1))
        pos[r, :k] = np.sort(rng.choice(np.arange(1, S), size=k, replace=False))
        mids[r, :k] = rng.integers(0, 30000, size=k)
    nsp = rng.integers(0, 2, size=n).astype(np.int8)
    h5.write_shard(path, ids, mask, seg, pos, mids, nsp, gzip)
    lab = np.full((n, S), -1, np.int64)
    for r in range(n):
        for j in range(P):
            if pos[r, j] == 0:
                break
            lab[r, pos[r, j]] = mids[r, j]
    return [ids.astype(np.int64), seg.astype(np.int64), mask.astype(np.int64), lab, nsp.astype(np.int64)]


def check_h5(h5, rng):
    S, P = 32, 5
    with tempfile.TemporaryDirectory() as d:
        sizes = [7, 1, 13]
        want = []
        shards = []
        for i, n in enumerate(sizes):
            p = os.path.join(d, "s%d.h5" % i)
            want.append(make_shard(h5, p, n, S, P, rng, gzip=i % 2))
            shards.append(h5.H5Shard(p, P))
            assert len(shards[-1]) == n and shards[-1].seq_len == S and shards[-1].num_pred == P
        full = [np.concatenate([w[k] for w in want]) for k in range(5)]
        N = sum(sizes)
        # read_rows into an offset of a larger buffer
        s0 = shards[2]
        bufs = [np.zeros((20, S), np.int64) for _ in range(4)] + [np.zeros(20, np.int64)]
        s0.read_rows(3, 9, *[b.ctypes.data for b in bufs], 5)
        for k in range(5):
            np.testing.assert_array_equal(bufs[k][5:14], want[2][k][3:12])
        try:
            s0.read_rows(10, 9, *[b.ctypes.data for b in bufs], 0)
            raise AssertionError("out-of-range read accepted")
        except IndexError:
            pass
        sset = h5.ShardSet(shards)
        assert len(sset) == N
        for _ in range(50):
            idx = rng.integers(0, N, size=int(rng.integers(1, 24))).astype(np.int64)
            out = [np.zeros((len(idx), S), np.int64) for _ in range(4)] + [np.zeros(len(idx), np.int64)]
            sset.gather(idx, *out)
            for k in range(5):
                np.testing.assert_array_equal(out[k], full[k][idx])
        # prefetcher over a shuffled epoch with a ring of 3 slots, 2 workers
        order = rng.permutation(N).astype(np.int64)
        batches = [order[i:i + 4] for i in range(0, N, 4)] + [np.zeros(0, np.int64)]
        slots = [[np.zeros((4, S), np.int64) for _ in range(4)] + [np.zeros(4, np.int64)] for _ in range(3)]
        pf = h5.Prefetcher(sset, batches, [[b.ctypes.data for b in s] for s in slots], 4, 2)
        seen = 0
        while True:
            slot, bsz = pf.next()
            if slot < 0:
                break
            b = batches[seen]
            assert bsz == len(b)
            for k in range(5):
                np.testing.assert_array_equal(slots[slot][k][:bsz], full[k][b])
            pf.release(slot)
            seen += 1
        assert seen == len(batches)
        pf.stop()
        # early stop with batches still in flight must not touch freed memory
        pf = h5.Prefetcher(sset, batches, [[b.ctypes.data for b in s] for s in slots], 4, 2)
        pf.next()
        pf.stop()
        del pf


def main():
    d = sys.argv[1]
    rng = np.random.default_rng(0)
    check_batcher(load("_native", d), rng)
    print("batcher ok")
    if os.path.exists(d) and any(f.startswith("_h5.") for f in os.listdir(d)):
        check_h5(load("_h5", d), rng)
        print("h5 ok")
    print("SANITIZERS CLEAN")


if __name__ == "__main__":
    main()
