"""Sparse exchange of the embedding tables' gradient (parallel/tied.py) on CPU / gloo, 2 ranks.

A toy model with the BERT structure of the tables: word / position / token-type tables looked up
by a Function that hands its rows to the engine (like FusedEmbedding), a decoder tied to the word
table whose backward accumulates its dense gradient into the flat buffer and signals the engine
(like FusedPreTrainingLoss), and an embedding LayerNorm-like module of its own.  Checks:

* the gradients equal the dense-bucket engine's (and the single-process sum over ranks),
  replicas identical, with and without a ``no_sync`` micro-batch before the synchronised one;
* the early bucket goes out before any backward work of the encoder's layers finishes and the
  only collectives after the embedding backward are the row gather (cap*H*4 bytes) and the
  embedding-rest bucket;
* micro-batches smaller than the agreed capacity are padded (padding keys skipped).
"""
import socket

import multiprocessing as mp
import pytest
import torch
import torch.distributed as dist

pytestmark = pytest.mark.slow

V, P, TV, H = 40, 16, 2, 8  # tables of whole 256-B blocks: adjacent in the flat buffer


class _Emb(torch.autograd.Function):
    @staticmethod
    def forward(ctx, ids, tt, word, pos, typ, store):
        from hetseq_amd.parallel import tied

        B, S = ids.shape
        ctx.save_for_backward(ids, tt)
        ctx.store = store
        ctx.tables = None
        h = tied.lookup(store.grad_view(word)) if store is not None else None
        if h is not None and h.begin(ids, tt, bool(ctx.needs_input_grad[2])):
            ctx.tables = h
        ctx.params = (word, pos, typ)
        return (word[ids] + pos[:S].unsqueeze(0) + typ[tt]).reshape(B * S, H)

    @staticmethod
    def backward(ctx, dy):
        ids, tt = ctx.saved_tensors
        B, S = ids.shape
        word, pos, typ = ctx.params
        if ctx.tables is not None:
            ctx.tables.row_buffer(B * S, H).copy_(dy)
            ctx.tables.rows_ready()
        else:
            st = ctx.store
            st.grad_view(word).index_add_(0, ids.reshape(-1), dy)
            st.grad_view(pos)[:S].add_(dy.view(B, S, H).sum(0))
            st.grad_view(typ).index_add_(0, tt.reshape(-1), dy)
        return None, None, None, None, None, None


class _TiedDecoder(torch.autograd.Function):
    @staticmethod
    def forward(ctx, h, word, store):
        ctx.save_for_backward(h, word)
        ctx.store = store
        return h @ word.t()

    @staticmethod
    def backward(ctx, dl):
        from hetseq_amd.parallel import tied

        h, word = ctx.saved_tensors
        view = ctx.store.grad_view(word)
        view.add_(dl.t() @ h)
        t = tied.lookup(view)
        if t is not None:
            t.dense_ready(dl.device)
        return dl @ word, None, None


class _Net(torch.nn.Module):
    def __init__(self):
        super().__init__()
        self.word = torch.nn.Parameter(torch.randn(V, H) * 0.3)
        self.pos = torch.nn.Parameter(torch.randn(P, H) * 0.3)
        self.typ = torch.nn.Parameter(torch.randn(TV, H) * 0.3)
        self.ln_w = torch.nn.Parameter(torch.ones(H))
        self.ln_b = torch.nn.Parameter(torch.zeros(H))
        self.l1 = torch.nn.Linear(H, H)
        self.l2 = torch.nn.Linear(H, H)
        self.store = None

    def sparse_embedding(self):
        return [self.word, self.pos, self.typ], [self.ln_w, self.ln_b]

    def forward(self, ids, tt, labels):
        x = _Emb.apply(ids, tt, self.word, self.pos, self.typ, self.store)
        x = x * self.ln_w + self.ln_b
        h = torch.tanh(self.l2(torch.tanh(self.l1(x))))
        logits = _TiedDecoder.apply(h, self.word, self.store)
        return torch.nn.functional.cross_entropy(logits, labels.reshape(-1), reduction="sum")


def _batch(rank, micro, B=3, S=5):
    g = torch.Generator().manual_seed(100 * rank + micro)
    ids = torch.randint(0, V, (B, S), generator=g)
    ids[0, :2] = 7  # a token shared by both ranks
    tt = torch.randint(0, TV, (B, S), generator=g)
    labels = torch.randint(0, V, (B, S), generator=g)
    return ids, tt, labels


def _worker(rank, port, q, sparse, micro_batches, small_last):
    try:
        _work(rank, port, q, sparse, micro_batches, small_last)
    except BaseException as e:  # report instead of leaving the parent waiting on the queue
        q.put((rank, None, repr(e), 0))
        raise


def _work(rank, port, q, sparse, micro_batches, small_last):
    from hetseq_amd.parallel.ddp import FlatDDP
    from hetseq_amd.runtime.flat import FlatParamStore

    dist.init_process_group("gloo", init_method="tcp://127.0.0.1:%d" % port, world_size=2, rank=rank)
    torch.manual_seed(0)
    net = _Net()
    store = FlatParamStore(net)
    net.store = store
    ddp = FlatDDP(net, store, bucket_cap_mb=0.0002, sparse_embedding=net.sparse_embedding() if sparse else None,
                  sparse_capacity=15 if small_last else None)
    if sparse:
        assert ddp.tables is not None
    store.grad.zero_()
    for micro in range(micro_batches):
        last = micro == micro_batches - 1
        ctx = torch.enable_grad() if last else ddp.no_sync()
        B = 2 if (small_last and last) else 3
        with ctx:
            ddp(*_batch(rank, micro, B=B)).backward()
    q.put((rank, store.grad.numpy().copy(), ddp.comm_log, len(ddp.buckets)))
    dist.destroy_process_group()


def _run(sparse, micro_batches=1, small_last=False):
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_worker, args=(r, port, q, sparse, micro_batches, small_last)) for r in range(2)]
    for p in procs:
        p.start()
    res = {}
    for _ in range(2):
        r, g, log, nb = q.get(timeout=120)
        assert g is not None, "rank %d failed: %s" % (r, log)
        res[r] = (torch.from_numpy(g), log, nb)
    for p in procs:
        p.join(60)
        assert p.exitcode == 0
    return res


def _reference(micro_batches, small_last=False):
    from hetseq_amd.runtime.flat import FlatParamStore

    total = None
    for rank in range(2):
        torch.manual_seed(0)
        net = _Net()
        st = FlatParamStore(net)
        net.store = st
        st.grad.zero_()
        for micro in range(micro_batches):
            B = 2 if (small_last and micro == micro_batches - 1) else 3
            net(*_batch(rank, micro, B=B)).backward()
        total = st.grad.clone() if total is None else total + st.grad
    return total


@pytest.mark.parametrize("micro_batches", [1, 2])
def test_sparse_tables_match_dense_engine(micro_batches):
    sp = _run(True, micro_batches)
    dn = _run(False, micro_batches)
    ref = _reference(micro_batches)
    g0, log, nb = sp[0]
    assert torch.equal(g0, sp[1][0])  # replicas identical
    assert torch.allclose(g0, dn[0][0], atol=1e-5, rtol=1e-5)
    assert torch.allclose(g0, ref, atol=1e-5, rtol=1e-5)
    names = [w for w, *_ in log]
    # keys in forward, the tables' dense bucket before every encoder bucket, rows after backward
    assert names[0] == "keys" and names[1] == "allreduce_tables", names
    tail = [(w, b) for w, b, t, _ in log if t]
    assert [w for w, _ in tail][0] == "rows", tail
    assert sum(b for w, b in tail if w == "rows") == 15 * H * 4  # B*S*H*4 per rank
    assert sum(r for w, _, t, r in log if t and w == "rows") == 15 * H * 4  # received: (W-1) x payload
    # at most the embedding LayerNorm's own bucket (two H-vectors, each padded to 256 B in the flat buffer)
    assert sum(b for w, b in tail if w != "rows") <= 2 * 256


def test_sparse_tables_pad_small_micro_batch():
    sp = _run(True, 1, small_last=True)
    ref = _reference(1, small_last=True)
    g0 = sp[0][0]
    assert torch.equal(g0, sp[1][0])
    assert torch.allclose(g0, ref, atol=1e-5, rtol=1e-5)
    rows = [b for w, b, *_ in sp[0][1] if w == "rows"]
    assert rows == [15 * H * 4]  # the agreed capacity, 10 real rows + 5 padding rows


def test_sparse_policy_by_world_size():
    """The sparse exchange is used only while its tail (the row all-gather, (W-1) x cap x H received
    per rank) is smaller than the dense bucket's all-reduce of the region (2(W-1)/W x K x H):
    BERT-base tables at 4,096 tokens per rank pay up to W = 15, not at 16; without a configured
    capacity the caller opted in."""
    from hetseq_amd.parallel.tied import SparseTableSync

    tables = [torch.empty(30522, 1), torch.empty(512, 1), torch.empty(2, 1)]
    assert SparseTableSync.pays(2, 4096, tables)
    assert SparseTableSync.pays(8, 4096, tables)
    assert SparseTableSync.pays(15, 4096, tables)
    assert not SparseTableSync.pays(16, 4096, tables)
    assert not SparseTableSync.pays(8, 8 * 4096, tables)  # seq 512 x 64 sentences per rank: dense
    assert SparseTableSync.pays(64, None, tables)


def test_received_bytes_accounting():
    """comm_log records what each rank RECEIVES: all-gather (W-1) x payload, ring all-reduce
    2(W-1)/W x payload; tail_bytes sums the received bytes of the collectives after backward."""
    from hetseq_amd.parallel.ddp import FlatDDP

    class _Fake(object):
        world_size = 8
        comm_log = []
        _in_tail = False

    f = _Fake()
    t = torch.empty(1000)
    FlatDDP._log(f, "keys", t, "allgather")
    f._in_tail = True
    FlatDDP._log(f, "rows", t, "allgather")
    FlatDDP._log(f, "allreduce_bucket9", t)
    assert f.comm_log[1] == ("rows", 4000, True, 7 * 4000)
    assert f.comm_log[2] == ("allreduce_bucket9", 4000, True, 2 * 7 * 4000 // 8)
    assert FlatDDP.tail_bytes(f) == 7 * 4000 + 7000
