"""Data-parallel equivalence on the real HIP kernels: two ranks on cuda:0, gloo as
the transport (dist.py stages device tensors through the host for gloo; production runs use
RCCL). The reference step is single-device (tower_code/v1_usertower_train.py:794-845), so the
contract is: the per-rank objectives of dist.contrastive_objective_dp summed over ranks, and
the bucket-reduced gradients (GradBucket hooks firing during backward), equal
TT.contrastive_losses / its gradients on the rank-major concatenated global batch; and the
item-range-sharded top-k (dist.retrieve_topk_sharded over the HIP rsx_retrieve_topk) is
bit-exact against the unsharded call."""
import os
import socket

import pytest
import torch
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _dp_worker(rank, world, port, q):
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import recsys_amd  # noqa: F401
        from recsys_amd import dist as D
        from recsys_amd import ops, synth
        from recsys_amd.tower_code import v1_usertower_train as TT
        from recsys_amd.tower_code.v1_refine_usertower import SASRecUserTower
        from tests.helpers import small_cfg, small_universe, to_dev
        dev = torch.device("cuda:0")
        torch.cuda.set_device(dev)
        res = {}
        for precision in ("fp32", "bf16x3"):
            ops.set_nce_precision(precision)
            cfg = small_cfg(num_items=500)
            items = small_universe(500)
            G = 64
            b = G // world
            full = to_dev(synth.make_batch(items, G, seed=31), dev)
            mine = {k: (v[rank * b:(rank + 1) * b] if torch.is_tensor(v) else v) for k, v in full.items()}
            lookup = items.pretrained.to(dev)

            def build():
                torch.manual_seed(0)
                m = SASRecUserTower(cfg).to(dev)
                m.train()
                it = TT.SASRecItemTower(500, 128, items.log_q.clone()).to(dev)
                it.init_from_pretrained(lookup)
                it.set_freeze_state(False)
                return m, it

            # single-GPU reference on the concatenated batch (own copy: no bucket hooks on it)
            m1, it1 = build()
            tot1, main1, cl1 = TT.contrastive_losses(m1, it1, it1.log_q, full, cfg, pretrained_lookup=lookup)
            tot1.backward()
            # this rank's share, gradients summed by the hooked buckets (several small buckets)
            m2, it2 = build()
            params = list(m2.parameters()) + list(it2.parameters())
            bucket = D.GradBucket(params, bucket_mb=0.25)
            assert len(bucket.buckets) > 2
            obj, tot, main, cl = D.contrastive_objective_dp(m2, it2, it2.log_q, mine, cfg, pretrained_lookup=lookup)
            obj.backward()
            launched_in_backward = bucket.launched
            bucket()
            for a, r in ((tot, tot1), (main, main1), (cl, cl1)):
                assert abs(a.item() - r.item()) < 1e-4, (precision, a.item(), r.item())
            worst = 0.0
            names = [n for n, _ in m2.named_parameters()] + ["item_matrix.weight"]
            for name, p_ref, p in zip(names, list(m1.parameters()) + list(it1.parameters()), params):
                g_ref = p_ref.grad if p_ref.grad is not None else torch.zeros_like(p_ref)
                assert p.grad is not None, name
                scale = g_ref.abs().max().item() + 1e-12
                err = (p.grad - g_ref).abs().max().item()
                assert err <= 2e-3 * scale + 1e-6, f"{precision} {name}: err {err} vs scale {scale}"
                worst = max(worst, err / scale)
            res[precision] = (round(worst, 7), launched_in_backward)

        # sharded exact top-k on the HIP kernel: dyadic inputs (exact fp32 dot products) with
        # ties planted across the shard boundary
        g = torch.Generator().manual_seed(5)
        corpus = (torch.randint(-8, 9, (3001, 128), generator=g).float() / 8.0)
        corpus[2500] = corpus[17]
        corpus[1600] = corpus[1400]
        queries = (torch.randint(-8, 9, (37, 128), generator=g).float() / 8.0)
        corpus, queries = corpus.to(dev), queries.to(dev)
        bounds = [0, 1501, 3001]
        lo, hi = bounds[rank], bounds[rank + 1]
        s, i = D.retrieve_topk_sharded(queries, corpus[lo:hi], lo, 100)
        s_ref, i_ref = ops.retrieve_topk(queries, corpus, 100)
        assert torch.equal(i.cpu(), i_ref.cpu())
        assert torch.equal(s.cpu(), s_ref.float().cpu())
        q.put((rank, "ok", res))
    except Exception as e:  # pragma: no cover - reported to the parent
        import traceback
        q.put((rank, repr(e) + traceback.format_exc()[-1500:], None))
    finally:
        dist.destroy_process_group()


def test_dp_objective_grads_and_sharded_topk_world2(gpu):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_dp_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    out = [q.get(timeout=110) for _ in procs]
    for p in procs:
        p.join(timeout=30)
    status = {r: s for r, s, _ in out}
    assert status == {0: "ok", 1: "ok"}, status
    # buckets were launched from the gradient hooks during backward, before the flush
    for _, _, res in out:
        for precision, (worst, launched) in res.items():
            assert launched >= 1, (precision, launched)


def _dp_fullsize_worker(rank, world, port, q, G=8192, precisions=("bf16x3", "fp32")):
    """Global batch G (8192: 2 x 4096; configs[3]'s 32,768: 2 x 16,384) split over the ranks (H&M-shaped lengths, 47,062 items: ~153k valid steps,
    ~24.4k distinct targets), so the grouped loss's column split, XCD remap and tail split run
    with FOREIGN columns (the other rank's targets, t_cols = the gathered ids) and user ids
    offset by rank * 4096 (dist.py prepare_step_index)."""
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import recsys_amd  # noqa: F401
        from recsys_amd import dist as D
        from recsys_amd import ops, synth
        from recsys_amd.tower_code import v1_usertower_train as TT
        from recsys_amd.tower_code.v1_refine_usertower import SASRecUserTower
        from tests.helpers import to_dev
        dev = torch.device("cuda:0")
        torch.cuda.set_device(dev)
        hs = synth.HASH_SIZE
        I = 47_062
        cfg = TT.PipelineConfig(num_items=I, num_prod_types=hs, num_colors=hs, num_graphics=hs, num_sections=hs,
                                dropout=0.0)
        items = synth.make_items(num_items=I, d=128, seed=0)
        b = G // world
        full = to_dev(synth.make_batch(items, G, seed=100), dev)
        mine = {k: (v[rank * b:(rank + 1) * b] if torch.is_tensor(v) else v) for k, v in full.items()}
        lookup = items.pretrained.to(dev)
        n_dist = int(torch.unique(full["target_ids"][~full["padding_mask"]]).numel())
        res = {"distinct_targets": n_dist}
        for precision in precisions:
            ops.set_nce_precision(precision)

            def build():
                torch.manual_seed(0)
                m = SASRecUserTower(cfg).to(dev)
                m.train()
                it = TT.SASRecItemTower(I, 128, items.log_q.clone()).to(dev)
                it.init_from_pretrained(lookup)
                it.set_freeze_state(False)
                return m, it

            m1, it1 = build()
            tot1, main1, cl1 = TT.contrastive_losses(m1, it1, it1.log_q, full, cfg, pretrained_lookup=lookup)
            tot1.backward()
            m2, it2 = build()
            params = list(m2.parameters()) + list(it2.parameters())
            bucket = D.GradBucket(params)
            obj, tot, main, cl = D.contrastive_objective_dp(m2, it2, it2.log_q, mine, cfg, pretrained_lookup=lookup)
            obj.backward()
            bucket()
            for a, r in ((tot, tot1), (main, main1), (cl, cl1)):
                assert abs(a.item() - r.item()) < 1e-4, (precision, a.item(), r.item())
            worst = 0.0
            names = [n for n, _ in m2.named_parameters()] + ["item_matrix.weight"]
            for name, p_ref, p in zip(names, list(m1.parameters()) + list(it1.parameters()), params):
                g_ref = p_ref.grad if p_ref.grad is not None else torch.zeros_like(p_ref)
                assert p.grad is not None, name
                scale = g_ref.abs().max().item() + 1e-12
                err = (p.grad - g_ref).abs().max().item()
                assert err <= 2e-3 * scale + 1e-6, f"{precision} {name}: err {err} vs scale {scale}"
                worst = max(worst, err / scale)
            res[precision] = (round(tot.item(), 6), round(tot1.item(), 6), round(worst, 7))
            del m1, it1, m2, it2, bucket, params, obj, tot1
            torch.cuda.empty_cache()
        q.put((rank, "ok", res))
    except Exception as e:  # pragma: no cover - reported to the parent
        import traceback
        q.put((rank, repr(e) + traceback.format_exc()[-1500:], None))
    finally:
        dist.destroy_process_group()


def test_dp_fullsize_world2_equals_single_gpu(gpu):
    """contrastive_objective_dp summed over 2 ranks (4096 users each) and the bucket-reduced
    gradients == TT.contrastive_losses / its gradients on the concatenated 8192-user batch
    (v1_usertower_train.py:794-845): loss 1e-4, every gradient 2e-3 of its scale, both precisions."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_dp_fullsize_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    out = [q.get(timeout=115) for _ in procs]
    for p in procs:
        p.join(timeout=30)
    status = {r: s for r, s, _ in out}
    assert status == {0: "ok", 1: "ok"}, status
    print({r: res for r, _, res in out})
    assert out[0][2]["distinct_targets"] >= 10_000


def test_dp_global_batch_32768_world2_equals_single_gpu(gpu):
    """configs[3]'s global batch: 2 ranks x 16,384 users (~600k valid steps, ~41k distinct
    targets, all-gathered ids so every rank's loss runs against the global pool) ==
    TT.contrastive_losses / its gradients on the concatenated 32,768-user batch on one device:
    loss 1e-4, every gradient 2e-3 of its scale (bf16x3, the step's precision)."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_dp_fullsize_worker, args=(r, 2, port, q, 32_768, ("bf16x3",))) for r in range(2)]
    for p in procs:
        p.start()
    out = [q.get(timeout=115) for _ in procs]
    for p in procs:
        p.join(timeout=30)
    status = {r: s for r, s, _ in out}
    assert status == {0: "ok", 1: "ok"}, status
    print({r: res for r, _, res in out})
    assert out[0][2]["distinct_targets"] >= 35_000


def _sharded_1m_worker(rank, world, port, q):
    """configs[4]'s corpus sharded by item range over 2 ranks (500,001 + 499,999 items): dyadic
    values (exact scores, heavy exact ties, some of them planted across the shard boundary),
    k = 100 and 500; the merged result is bit-identical to the unsharded call and the oracle."""
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import recsys_amd  # noqa: F401
        from recsys_amd import dist as D
        from recsys_amd import ops
        from oracle import retrieval as OR
        dev = torch.device("cuda:0")
        torch.cuda.set_device(dev)
        g = torch.Generator().manual_seed(51)
        NI = 1_000_000
        corpus = torch.randint(-4, 5, (NI, 128), generator=g).float() / 8.0
        queries = torch.randint(-4, 5, (64, 128), generator=g).float() / 8.0
        corpus[500_001] = corpus[17]
        corpus[499_999] = corpus[900_000]
        bounds = [0, 500_001, NI]
        lo, hi = bounds[rank], bounds[rank + 1]
        cd, qd = corpus.to(dev), queries.to(dev)
        for k in (100, 500):
            s, i = D.retrieve_topk_sharded(qd, cd[lo:hi], lo, k)
            s_ref, i_ref = ops.retrieve_topk(qd, cd, k)
            assert torch.equal(i.cpu(), i_ref.cpu()), k
            assert torch.equal(s.cpu(), s_ref.float().cpu()), k
            if rank == 0:
                rs, ri = OR.retrieve_topk_chunked(queries, corpus, k)
                assert torch.equal(i.cpu(), ri) and torch.equal(s.cpu().double(), rs), k
        q.put((rank, "ok", None))
    except Exception as e:  # pragma: no cover - reported to the parent
        import traceback
        q.put((rank, repr(e) + traceback.format_exc()[-1500:], None))
    finally:
        dist.destroy_process_group()


def test_sharded_topk_1m_world2_bit_exact(gpu):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_sharded_1m_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    out = [q.get(timeout=115) for _ in procs]
    for p in procs:
        p.join(timeout=30)
    status = {r: s for r, s, _ in out}
    assert status == {0: "ok", 1: "ok"}, status
