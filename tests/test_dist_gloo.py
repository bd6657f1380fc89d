"""world_size-2 gloo (CPU) tests of the data-parallel plumbing in dist.py: variable-length
all-gathers, the autograd all-gather of user vectors, the gradient bucket, and the
sum-over-local-rows / global-count decomposition of the contrastive objective (evaluated with
the dense CPU restatement, the same math the HIP kernels compute per rank)."""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp
import torch.nn.functional as F


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _dense_rows_loss(A, B, off, tau=0.1):
    """sum_i CE(A_i B^T / tau, label i + off) over this shard's rows."""
    S = A @ B.T / tau
    lab = torch.arange(A.shape[0]) + off
    return F.cross_entropy(S, lab, reduction="sum")


def _worker(rank, world, port, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import recsys_amd  # noqa: F401
        from recsys_amd import dist as D
        # variable-length gather
        n = 3 + rank * 2
        x = torch.arange(n, dtype=torch.int64) + 100 * rank
        counts = D.all_gather_counts(n, "cpu")
        got = D.all_gather_var(x, counts)
        exp = torch.cat([torch.arange(3 + r * 2) + 100 * r for r in range(world)])
        assert counts == [3 + 2 * r for r in range(world)]
        assert torch.equal(got, exp)
        # the background index builder is single-rank only (its all-gathers would leave program order)
        try:
            D.IndexPrefetcher()
            raise AssertionError("IndexPrefetcher must refuse world > 1")
        except RuntimeError:
            pass

        # decomposition of a two-view InfoNCE over a global batch of 8 users
        g = torch.Generator().manual_seed(0)
        Wt = torch.randn(16, 128, generator=g)
        X1 = torch.randn(8, 16, generator=g)
        X2 = X1 + 0.1 * torch.randn(8, 16, generator=g)
        b = 8 // world
        w_loc = Wt.clone().requires_grad_()
        # hook-driven buckets (~1 KB each: several buckets, launched during backward); `unused`
        # gets no gradient on any rank (stays None), `partial` only on rank 0 (summed anyway)
        unused = torch.zeros(5, requires_grad=True)
        partial = torch.ones(300, requires_grad=True)
        bias = torch.zeros(128, requires_grad=True)
        bucket = D.GradBucket([w_loc, unused, partial, bias], bucket_mb=1e-3)
        assert len(bucket.buckets) > 2
        for step in range(2):   # the second step reuses the buckets
            for p in (w_loc, unused, partial, bias):
                p.grad = None
            z1 = F.normalize(X1[rank * b:(rank + 1) * b] @ w_loc + bias, dim=1)
            z2 = F.normalize(X2[rank * b:(rank + 1) * b] @ w_loc + bias, dim=1)
            z2_glob = D.all_gather_rows(z2, [b] * world)
            obj = _dense_rows_loss(z1, z2_glob, rank * b) / 8.0
            if rank == 0:
                obj = obj + partial.square().sum()
            obj.backward()
            bucket()
        total = obj.detach().clone()
        D.all_reduce_sum_(total)
        # single-process reference
        w_ref = Wt.clone().requires_grad_()
        b_ref = torch.zeros(128, requires_grad=True)
        ref = _dense_rows_loss(F.normalize(X1 @ w_ref + b_ref, dim=1), F.normalize(X2 @ w_ref + b_ref, dim=1),
                               0) / 8.0
        ref.backward()
        torch.testing.assert_close(total, ref.detach() + 300.0, atol=1e-5, rtol=1e-6)
        torch.testing.assert_close(w_loc.grad, w_ref.grad, atol=1e-6, rtol=1e-5)
        torch.testing.assert_close(bias.grad, b_ref.grad, atol=1e-6, rtol=1e-5)
        assert unused.grad is None
        torch.testing.assert_close(partial.grad, torch.full((300,), 2.0))

        # gradient accumulation: micro-batch 0 under no_sync, micro-batch 1 synchronising; the
        # parameter listed twice is bucketed once; `late` gets a gradient only in micro-batch 0
        # (its hook never fires in the synchronising pass, bucket() copies it in)
        w2 = Wt.clone().requires_grad_()
        late = torch.ones(7, requires_grad=True)
        acc = D.GradBucket([w2, late, w2], bucket_mb=1e-3)
        assert len(acc.params) == 2
        Xs = [X1[rank * b:(rank + 1) * b], X2[rank * b:(rank + 1) * b]]
        with acc.no_sync():
            (Xs[0] @ w2).square().sum().backward()
            (late * (rank + 1)).sum().backward()
        (Xs[1] @ w2).square().sum().backward()
        acc()
        w_ref2 = Wt.clone().requires_grad_()
        ((X1 @ w_ref2).square().sum() + (X2 @ w_ref2).square().sum()).backward()
        torch.testing.assert_close(w2.grad, w_ref2.grad, atol=1e-4, rtol=1e-5)
        torch.testing.assert_close(late.grad, torch.full((7,), float(sum(r + 1 for r in range(world)))))
        # two synchronising backward passes before bucket() is a usage error, not silent divergence
        w2.grad = None
        (Xs[0] @ w2).sum().backward()
        try:
            (Xs[1] @ w2).sum().backward()
            raise AssertionError("second backward was accepted")
        except RuntimeError as e:
            assert "second gradient" in str(e)
        acc._reset()
        q.put((rank, "ok"))
    except Exception as e:  # pragma: no cover - reported to the parent
        q.put((rank, repr(e)))
    finally:
        dist.destroy_process_group()


def test_dp_plumbing_world2_gloo():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=120) for _ in procs)
    for p in procs:
        p.join(timeout=60)
    assert res == {0: "ok", 1: "ok"}, res


def _retrieval_worker(rank, world, port, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import recsys_amd  # noqa: F401
        from recsys_amd import dist as D
        from oracle.retrieval import retrieve_topk as ref_topk
        g = torch.Generator().manual_seed(3)
        corpus = torch.randn(1001, 128, generator=g)
        corpus[700] = corpus[10]               # exact tie across shards: lower index must win
        queries = torch.randn(6, 128, generator=g)
        bounds = [0, 523, 1001]
        lo, hi = bounds[rank], bounds[rank + 1]

        def local(qv, items, k):
            s, i = ref_topk(qv, items, k)
            return s.float(), i

        s, i = D.retrieve_topk_sharded(queries, corpus[lo:hi], lo, 50, local_topk=local)
        s_ref, i_ref = ref_topk(queries, corpus, 50)
        assert torch.equal(i, i_ref), (i[0, :10], i_ref[0, :10])
        torch.testing.assert_close(s, s_ref.float())
        q.put((rank, "ok"))
    except Exception as e:  # pragma: no cover - reported to the parent
        q.put((rank, repr(e)))
    finally:
        dist.destroy_process_group()


def test_sharded_retrieval_merge_gloo():
    """Item-range sharded top-k: per-shard top-k with global indices,
    all-gather, (score desc, index asc) merge == top-k over the whole corpus."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_retrieval_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in ps:
        p.start()
    res = dict(q.get(timeout=120) for _ in ps)
    for p in ps:
        p.join(timeout=60)
    assert res == {0: "ok", 1: "ok"}, res
