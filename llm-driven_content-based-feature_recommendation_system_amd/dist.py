"""Data-parallel contrastive step over RCCL (torch.distributed backend "nccl" on ROCm).

The reference is single-device; this is the MI355X-native multi-GPU form of
train_user_tower_all_time (tower_code/v1_usertower_train.py:717-893) whose result equals the
single-GPU step on the rank-major concatenated global batch:

  * each rank owns a contiguous slice of the global batch's users and runs both tower
    views locally;
  * the main LogQ loss needs every rank's target *ids* as columns. The item matrix is
    replicated, so each rank rebuilds the normalised global column pool from the gathered
    ids itself: one all-gather of ids (~8 B/step-position) instead of 512 B embeddings;
  * DuoRec needs the other ranks' user vectors: the L2-normalised last-step vectors z1/z2
    are all-gathered (autograd-aware: their gradients are all-reduced back to the owners);
  * every loss is a sum over local rows divided by the GLOBAL row count, so the per-rank
    objectives add up to the single-GPU objective, and the replicated parameters' gradients
    are summed by bucketed all-reduces launched from gradient hooks during backward
    (GradBucket), finished before clipping;
  * the data-dependent step index (row counts, target ids) is exchanged over a second
    communicator (index_group) from the prefetch stream, ahead of the step that uses it.
Only the collective helpers here are device-agnostic (gloo-tested on CPU); the losses call
the HIP kernels through ops.
"""
from __future__ import annotations

import contextlib
import os

import torch
import torch.distributed as dist

from . import _native as N
from . import ops


_LOCAL_ONLY = False


def world():
    if not _LOCAL_ONLY and dist.is_available() and dist.is_initialized():
        return dist.get_rank(), dist.get_world_size()
    return 0, 1


@contextlib.contextmanager
def local_only():
    """Inside, this process behaves as a single-GPU run (world() == (0, 1): no collectives, no
    bucket exchange) although a process group exists: e.g. one rank timing the 1-GPU baseline of
    a strong-scaling measurement while the other ranks wait at a barrier."""
    global _LOCAL_ONLY
    prev, _LOCAL_ONLY = _LOCAL_ONLY, True
    try:
        yield
    finally:
        _LOCAL_ONLY = prev


def _host_staged(t: torch.Tensor, group=None) -> bool:
    """gloo carries device tensors only for some collectives: stage them through host memory
    (the CPU test transport; production runs use RCCL, which takes device pointers)."""
    return t.is_cuda and dist.get_backend(group) == "gloo"


def all_gather_into(bufs, t: torch.Tensor, group=None) -> None:
    if _host_staged(t, group):
        cb = [torch.empty(t.shape, dtype=t.dtype) for _ in bufs]
        dist.all_gather(cb, t.cpu(), group=group)
        for b, c in zip(bufs, cb):
            b.copy_(c)
        return
    dist.all_gather(bufs, t, group=group)


def all_reduce_(t: torch.Tensor, op=None, group=None, async_op=False):
    """In-place all-reduce (sum by default). Returns the work handle when async_op and the
    transport is asynchronous, else None."""
    op = dist.ReduceOp.SUM if op is None else op
    if _host_staged(t, group):
        c = t.cpu()
        dist.all_reduce(c, op=op, group=group)
        t.copy_(c)
        return None
    return dist.all_reduce(t, op=op, group=group, async_op=async_op)


_INDEX_GROUP = None


def index_group():
    """A second communicator for the step-index exchanges (row counts, target ids). Under RCCL
    each communicator has its own stream, so the next batch's index exchange, issued from the
    prefetch side stream while the current step runs, never queues behind that step's gradient
    all-reduce. Created lazily; every rank reaches the first call at the same point."""
    global _INDEX_GROUP
    if _INDEX_GROUP is None:
        _INDEX_GROUP = dist.new_group(backend=dist.get_backend())
    return _INDEX_GROUP


def all_gather_counts(n: int, device, group=None) -> list:
    """Every rank's local row count (one tiny all-gather + host read). Called only while a
    StepIndex is built (ahead of the step, on the prefetch stream, over index_group())."""
    rank, ws = world()
    if ws == 1:
        return [int(n)]
    t = torch.tensor([int(n)], device=device, dtype=torch.int64)
    out = [torch.empty_like(t) for _ in range(ws)]
    all_gather_into(out, t, group=group)
    return torch.cat(out).tolist()


def all_gather_var(x: torch.Tensor, counts: list, group=None) -> torch.Tensor:
    """Concatenate every rank's x[:counts[r]] (rank-major). Not differentiable."""
    rank, ws = world()
    if ws == 1:
        return x
    mx = max(counts)
    pad = torch.zeros((mx,) + tuple(x.shape[1:]), device=x.device, dtype=x.dtype)
    pad[: x.shape[0]] = x
    bufs = [torch.empty_like(pad) for _ in range(ws)]
    all_gather_into(bufs, pad, group=group)
    return torch.cat([b[:c] for b, c in zip(bufs, counts)], dim=0)


class _AllGatherRows(torch.autograd.Function):
    """Rank-major all-gather of [n_r, D] rows; backward sums every rank's gradient of the
    gathered matrix and returns this rank's slice (the reduce half of the exchange)."""

    @staticmethod
    def forward(ctx, x, counts):
        rank, _ = world()
        ctx.lo = sum(counts[:rank])
        ctx.n = counts[rank]
        return all_gather_var(x.contiguous(), counts)

    @staticmethod
    def backward(ctx, g):
        g = g.contiguous()
        if world()[1] > 1:
            all_reduce_(g)
        return g[ctx.lo: ctx.lo + ctx.n], None


def all_gather_rows(x: torch.Tensor, counts: list) -> torch.Tensor:
    if world()[1] == 1:
        return x
    return _AllGatherRows.apply(x, counts)


def all_reduce_sum_(t: torch.Tensor) -> torch.Tensor:
    if world()[1] > 1:
        all_reduce_(t)
    return t


class GradBucket:
    """Sum of the replicated parameters' gradients over ranks (DDP semantics), overlapped with
    backward. Parameters (deduplicated by identity) are grouped into ~bucket_mb buckets in
    reverse registration order (the order backward produces them); a post-accumulate-grad hook
    copies each gradient into its bucket's flat fp32 buffer, and a bucket's all-reduce is
    launched (asynchronously, on the communicator's stream) as soon as it and every earlier
    bucket are complete, so the exchange runs under the rest of backward. Launch order is the
    bucket index on every rank. Each bucket carries one has-gradient flag per parameter in the
    same buffer: after the exchange a parameter whose gradient is None on EVERY rank stays None
    (the single-GPU step's AdamW skips it), otherwise its gradient becomes the summed slice (a
    view of the bucket). Call the bucket after backward to launch what is left and wait.

    Contract: ONE synchronising backward per call. A second hook for the same parameter before
    the call raises (its bucket may already be in flight). Gradient accumulation runs the
    earlier micro-batches inside ``with bucket.no_sync():`` (hooks idle, p.grad accumulates),
    then the last backward outside it: its hooks copy the accumulated gradients."""

    def __init__(self, params, bucket_mb: float = 16.0):
        seen, self.params = set(), []
        for p in params:
            if p.requires_grad and id(p) not in seen:
                seen.add(id(p))
                self.params.append(p)
        self.numel = sum(p.numel() for p in self.params)
        cap = max(1, int(bucket_mb * (1 << 20) / 4))
        self.buckets = []          # [[param index, ...], ...]
        cur, size = [], 0
        for i in reversed(range(len(self.params))):
            n = self.params[i].numel()
            if cur and size + n > cap:
                self.buckets.append(cur)
                cur, size = [], 0
            cur.append(i)
            size += n
        if cur:
            self.buckets.append(cur)
        self.where = {}            # param index -> (bucket, offset, slot)
        self.sizes = []
        for b, idx in enumerate(self.buckets):
            o = 0
            for s, i in enumerate(idx):
                self.where[i] = (b, o, s)
                o += self.params[i].numel()
            self.sizes.append(o)
        self.flat = None
        self.by_id = {id(p): i for i, p in enumerate(self.params)}
        self.handles = [p.register_post_accumulate_grad_hook(self._on_grad) for p in self.params]
        self._sync = True
        self._reset()

    def _reset(self):
        self.filled = [0] * len(self.buckets)
        self.got = [False] * len(self.params)
        self.work = [None] * len(self.buckets)
        self.launched = 0
        self.active = False

    @contextlib.contextmanager
    def no_sync(self):
        """Backward passes inside accumulate into p.grad without touching the buckets."""
        prev, self._sync = self._sync, False
        try:
            yield
        finally:
            self._sync = prev

    def _buffers(self, dev):
        if self.flat is None or self.flat[0].device != dev:
            # [bucket values..., one has-grad flag per parameter]
            self.flat = [torch.empty(n + len(idx), device=dev, dtype=torch.float32)
                         for n, idx in zip(self.sizes, self.buckets)]
        return self.flat

    def _activate(self, dev):
        if not self.active:
            self.active = True
            for f, n in zip(self._buffers(dev), self.sizes):
                f[n:].zero_()

    def _copy_in(self, i):
        p = self.params[i]
        b, o, s = self.where[i]
        f = self.flat[b]
        f[o:o + p.numel()].copy_(p.grad.reshape(-1))
        f[self.sizes[b] + s].fill_(1.0)
        self.got[i] = True
        self.filled[b] += 1

    def _on_grad(self, p):
        if world()[1] == 1 or not self._sync:
            return
        i = self.by_id[id(p)]
        if self.got[i]:
            raise RuntimeError("GradBucket: a second gradient for one parameter before bucket() was called "
                               "(two backward passes?); accumulate earlier passes under bucket.no_sync()")
        self._activate(p.device)
        self._copy_in(i)
        while self.launched < len(self.buckets) and self.filled[self.launched] == len(self.buckets[self.launched]):
            self._launch(self.launched)

    def _launch(self, b):
        self.work[b] = all_reduce_(self.flat[b], async_op=True)
        self.launched += 1

    def __call__(self):
        if world()[1] == 1 or not self.params:
            return
        self._activate(self.params[0].device)
        # buckets still open: gradients whose hook did not fire in the last backward (made
        # under no_sync only) are copied now; parameters without a gradient contribute zeros
        for b in range(self.launched, len(self.buckets)):
            f = self.flat[b]
            for i in self.buckets[b]:
                if self.got[i]:
                    continue
                p = self.params[i]
                if p.grad is not None:
                    self._copy_in(i)
                else:
                    _, o, _ = self.where[i]
                    f[o:o + p.numel()].zero_()
        while self.launched < len(self.buckets):
            self._launch(self.launched)
        for b, w in enumerate(self.work):
            if w is not None:
                w.wait()
        for b, idx in enumerate(self.buckets):
            f = self.flat[b]
            flags = f[self.sizes[b]:]
            has = (flags > 0).tolist() if any(self.params[i].grad is None for i in idx) else None
            for s, i in enumerate(idx):
                p = self.params[i]
                _, o, _ = self.where[i]
                if p.grad is None and not (has and has[s]):
                    continue
                p.grad = f[o:o + p.numel()].view_as(p)
        self._reset()


class StepIndex:
    """Every data-dependent structure of one DP step (nothing depends on model state): the
    packed token sets and per-token inputs (v1_usertower_train.pack_inputs), the global row
    counts, the main loss's grouped-target index and the DuoRec keys."""


class _Packed:
    """PackedTokens' attributes for the device-built index (tower_code.v1_refine_usertower)."""

    def take(self, t: torch.Tensor) -> torch.Tensor:
        return t.reshape((-1,) + tuple(t.shape[2:]))[self.flat]


# RSX_DEVICE_INDEX=0: the torch builders (PackedTokens / pack_inputs / sort_segments /
# TargetGroups, ~12 host size queries per batch) instead of rsx_step_index_* (one host read)
_DEVICE_INDEX = os.environ.get("RSX_DEVICE_INDEX", "1") != "0"


def static_inputs(batch):
    """The per-user static inputs of the step: the nine id columns (int64) and cont_feats, NOT
    doubled for the two dropout views -- the static-profile program reads user r % B for output
    row r (ops.static_profile rows = 2B)."""
    from .tower_code.v1_usertower_train import _STATIC_KEYS
    return [batch[k].reshape(-1).to(torch.int64) for k in _STATIC_KEYS[:9]] + [batch[_STATIC_KEYS[9]]]


_ELEM = {torch.int64: 8, torch.int32: 4, torch.float32: 4, torch.uint8: 1}


def _carve(specs, dev):
    """Uninitialised tensors ((shape, dtype) per entry, None -> None) carved from one uint8
    allocation at 256-B aligned offsets (one allocator call instead of one per array)."""
    sizes, total = [], 0
    for sp in specs:
        if sp is None:
            sizes.append(None)
            continue
        shape, dt = sp
        n = 1
        for d in shape:
            n *= d
        nb = n * _ELEM[dt]
        sizes.append((total, nb))
        total += (nb + 255) // 256 * 256
    buf = torch.empty(max(total, 256), device=dev, dtype=torch.uint8)
    out = []
    for sp, sz in zip(specs, sizes):
        if sp is None:
            out.append(None)
            continue
        o, nb = sz
        out.append(buf[o:o + nb].view(sp[1]).view(sp[0]))
    return out


def _prepare_step_index_device(batch, pretrained_vecs, pretrained_lookup, n_items) -> StepIndex:
    """prepare_step_index on rsx_step_index_* (csrc/step_index.hip): the same arrays in the same
    orders as the torch builders, with ONE host read (the totals) per batch; at world > 1 the
    ranks exchange fixed-size [B*L + 1] target blocks, so no size is needed before the exchange."""
    from .tower_code.v1_usertower_train import _SEQ_ID_KEYS, _STATIC_KEYS

    lib = N.lib()
    rank, ws = world()
    pm = batch["padding_mask"]
    B, L = pm.shape
    dev = pm.device
    pm8 = ops._c(pm).view(torch.uint8) if pm.dtype == torch.bool else ops._c(pm.to(torch.uint8))
    tgt = ops._c(batch["target_ids"].to(torch.int64))
    seq = [ops._c(batch[k].to(torch.int64)) for k in _SEQ_ID_KEYS]
    nb = lib.rsx_step_index_workspace_bytes(B, L, n_items)
    wsb = torch.empty(nb, device=dev, dtype=torch.uint8)
    tloc = torch.empty(B * L + 1, device=dev, dtype=torch.int32)
    N.check(lib.rsx_step_index_count(N.ptr(pm8), N.ptr(tgt), N.ptr(seq[0]), B, L, n_items, N.ptr(wsb), nb,
                                     N.ptr(tloc), N.stream()), "step_index_count")
    if ws > 1:
        tglob = torch.empty(ws, B * L + 1, device=dev, dtype=torch.int32)
        all_gather_into(list(tglob.unbind(0)), tloc, group=index_group())
    else:
        tglob = tloc
    totals = torch.empty(8 + ws, device=dev, dtype=torch.int64)
    N.check(lib.rsx_step_index_totals(N.ptr(tglob), ws, B, L, n_items, N.ptr(wsb), nb, N.ptr(totals), N.stream()),
            "step_index_totals")
    tot = totals.tolist()  # the one host read
    T, Nr, D, E, U, C, err = tot[:7]
    if err:
        raise IndexError(f"step index: a target / item id outside [0, {n_items})")
    i64, i32, u8, f32 = torch.int64, torch.int32, torch.uint8, torch.float32
    specs = [((T,), i64), ((T,), i64), ((T,), i64), ((T,), u8), ((B + 1,), i32), ((B + 1,), i64), ((Nr,), i64),
             ((B,), i64), ((2 * T,), i64), ((2 * T,), i64), ((2 * T,), i64), ((2 * T,), u8), ((2 * B + 1,), i32),
             ((2 * B + 1,), i64), ((6, 2 * T), i64), (((2 * T, 128), f32) if pretrained_vecs is None else None),
             ((2 * T,), i64), ((C + 1,), i64), ((C,), i64), ((U + 1,), i64), ((U,), i64), ((D,), i64), ((D,), f32),
             ((Nr,), i32), ((Nr,), i32), ((Nr,), i32), ((Nr,), i32), ((E,), i32), ((E,), i32), ((E,), i32),
             ((D,), i32), ((D,), i32), ((B,), i32)]
    out = _carve(specs, dev)  # the 33 index arrays out of ONE allocation
    lk = ops._c(pretrained_lookup) if pretrained_vecs is None else None
    N.check(lib.rsx_step_index_fill(N.ptr(pm8), N.ptr(tgt), N.ptr_array(seq), N.ptr(lk),
                                    lk.stride(0) if lk is not None else 0, B, L, n_items,
                                    N.i64_array([T, Nr, D, E, U, C]), N.ptr(wsb), nb, N.ptr_array(out), N.stream()),
            "step_index_fill")
    pk, pk2 = _Packed(), _Packed()
    pk.flat, pk.tok_user, pk.tok_pos, pk.tok_pad, pk.seg_off, pk.seg_off64, pk.valid_tok, pk.last_tok = out[:8]
    pk.B, pk.L = B, L
    (pk2.flat, pk2.tok_user, pk2.tok_pos, pk2.tok_pad, pk2.seg_off, pk2.seg_off64) = out[8:14]
    pk2.B, pk2.L = 2 * B, L
    pk2.item_seg = tuple(out[16:21])
    tok_ids = list(out[14].unbind(0))
    if pretrained_vecs is None:
        pv_tok = out[15]
    else:
        pv_tok = pk.take(pretrained_vecs)
        pv_tok = torch.cat([pv_tok, pv_tok])
    static = static_inputs(batch)
    ix = StepIndex()
    ix.packed = (pk, pk2, tok_ids, pv_tok, static)
    ix.B = B
    ix.counts = [int(c) for c in tot[8:8 + ws]]
    ix.n_glob = sum(ix.counts)
    ix.groups = None
    if ix.n_glob > 0:
        ix.groups = ops.TargetGroups.from_arrays(*out[21:32], n_rows=Nr)
    ix.last_t = out[32]
    ix.t_glob_last = all_gather_var(ix.last_t, [B] * ws, group=index_group() if ws > 1 else None)
    ix.wsb = wsb  # keeps the workspace alive with the index (stream-ordered reuse)
    return ix


def _device_lookup_ok(pretrained_vecs, lookup, device) -> bool:
    """The device builder gathers the pretrained rows itself (si_pv_k: fp32 rows of exactly 128
    columns, read through a device pointer, no autograd). Any other lookup -- on the host, of
    another dtype or width, or one that requires grad -- takes the torch builders, whose
    ops.gather_rows handles those (and carries the gradient)."""
    if pretrained_vecs is not None:
        return True
    return (lookup is not None and lookup.device == device and lookup.dtype == torch.float32 and lookup.dim() == 2
            and lookup.shape[1] == 128 and lookup.stride(1) == 1 and not lookup.requires_grad)


def prepare_step_index(batch, pretrained_vecs=None, pretrained_lookup=None, n_items=None) -> StepIndex:
    """Builds the StepIndex of `batch` on the current stream. Device batches (L <= 64) use
    rsx_step_index_* (one host read: the totals); otherwise, or with RSX_DEVICE_INDEX=0, the torch
    builders, whose size queries (nonzero / unique / the count all-gather) each synchronise the
    host with that stream. n_items: the id domain (default: the pretrained lookup's rows)."""
    from .tower_code.v1_usertower_train import pack_inputs

    if n_items is None and pretrained_lookup is not None:
        n_items = pretrained_lookup.shape[0]
    if (_DEVICE_INDEX and n_items is not None and batch["item_ids"].is_cuda
            and batch["padding_mask"].shape[1] <= 64 and _device_lookup_ok(pretrained_vecs, pretrained_lookup,
                                                                          batch["item_ids"].device)):
        return _prepare_step_index_device(batch, pretrained_vecs, pretrained_lookup, int(n_items))
    rank, ws = world()
    device = batch["item_ids"].device
    B = batch["item_ids"].shape[0]
    target_ids = batch["target_ids"]
    ix = StepIndex()
    ix.packed = pack_inputs(batch, pretrained_vecs, pretrained_lookup)
    pk = ix.packed[0]
    ix.B = B
    grp = index_group() if ws > 1 else None
    ix.counts = all_gather_counts(pk.valid_tok.numel(), device, group=grp)
    ix.n_glob = sum(ix.counts)
    ix.groups = None
    if ix.n_glob > 0:
        t_loc = target_ids.reshape(-1)[pk.flat[pk.valid_tok]]
        user_loc = pk.tok_user[pk.valid_tok] + rank * B
        t_glob = all_gather_var(t_loc, ix.counts, group=grp)
        ix.groups = ops.TargetGroups(t_loc, user_loc, t_cols=t_glob)
    ix.last_t = target_ids.reshape(-1)[pk.flat[pk.last_tok]].to(torch.int32)  # the SupCon keys (as rsx_step_index_fill)
    ix.t_glob_last = all_gather_var(ix.last_t, [B] * ws, group=grp)
    return ix


_PREP_STREAM = None


def prepare_step_index_async(batch, pretrained_vecs=None, pretrained_lookup=None):
    """prepare_step_index on a high-priority side stream: its host synchronisations wait only
    for that stream's few small kernels, so calling it right after a step has been enqueued
    overlaps the next batch's index building (and its size queries) with the running step.
    The batch tensors must not be written by pending work. Pass the result to
    contrastive_step_dp(..., index=...), which orders the main stream after it."""
    global _PREP_STREAM
    if _PREP_STREAM is None:
        # RSX_INDEX_PRIORITY (A/B): the side stream's priority (-1 high, the default; 0 normal)
        _PREP_STREAM = torch.cuda.Stream(priority=int(os.environ.get("RSX_INDEX_PRIORITY", "-1")))
    with torch.cuda.stream(_PREP_STREAM):
        ix = prepare_step_index(batch, pretrained_vecs, pretrained_lookup)
        ix.ready = torch.cuda.Event()
        ix.ready.record(_PREP_STREAM)
    return ix


class IndexPrefetcher:
    """prepare_step_index_async on one background host thread: the index's host
    synchronisations (size queries behind the side stream's kernels, which wait for CU slots
    while the step's loss kernels hold the whole chip) then block that thread instead of the
    thread enqueueing the steps, so the main stream's queue never runs dry waiting for them.
    One worker: indexes are built in submission order. Single-rank only — with several ranks
    the index all-gathers (index_group) must stay in program order with the step's collectives."""

    def __init__(self):
        import concurrent.futures
        if world()[1] > 1:
            raise RuntimeError("IndexPrefetcher is single-rank only (use prepare_step_index_async with several ranks)")
        self._ex = concurrent.futures.ThreadPoolExecutor(max_workers=1, thread_name_prefix="rsx-index")
        self._pending = {}

    def submit(self, key, batch, pretrained_vecs=None, pretrained_lookup=None):
        dev = torch.cuda.current_device()

        def work():
            torch.cuda.set_device(dev)
            return prepare_step_index_async(batch, pretrained_vecs, pretrained_lookup)

        self._pending[key] = self._ex.submit(work)

    def pop(self, key):
        fut = self._pending.pop(key, None)
        return None if fut is None else fut.result()

    def close(self):
        for fut in self._pending.values():
            fut.result()
        self._pending.clear()
        self._ex.shutdown(wait=True)


_HELD = []          # (index, event): adopted indexes kept alive until the consuming stream passed them
_LAST_ADOPTED = None


def _adopt(ix):
    """Order the current stream after an async-prepared index and keep its memory alive for it.

    The index's tensors were allocated on the prefetch stream, so once freed the caching allocator
    may hand their blocks to that stream's next index while this stream's kernels of the step still
    read them. Instead of a record_stream per tensor (~40 per index), the adopted index itself is held
    until an event recorded on this stream at the NEXT adoption -- after all of its step's work --
    has completed; then it is released."""
    global _LAST_ADOPTED
    ev = getattr(ix, "ready", None)
    if ev is None:
        return
    cur = torch.cuda.current_stream()
    cur.wait_event(ev)
    ix.ready = None
    if _LAST_ADOPTED is not None:
        done = torch.cuda.Event()
        done.record(cur)
        _HELD.append((_LAST_ADOPTED, done))
    _LAST_ADOPTED = ix
    while _HELD and _HELD[0][1].query():
        _HELD.pop(0)


def release_held_indexes(sync=True):
    """Drop the indexes _adopt keeps alive (end of training); sync: wait for the device first."""
    global _LAST_ADOPTED
    if sync and torch.cuda.is_available():
        torch.cuda.synchronize()
    _HELD.clear()
    _LAST_ADOPTED = None


def contrastive_objective_dp(model, item_tower, log_q_tensor, batch, cfg, pretrained_lookup=None,
                             pretrained_vecs=None, temperature=0.1, index=None):
    """This rank's share of the global objective (reference :787-845 on the global batch).

    batch holds this rank's users (global user index = rank * B_local + b). index: a
    StepIndex of this batch prepared ahead (prepare_step_index[_async]); built here if None.
    Returns (local objective to backward, global total / main / cl for logging; the
    logging values are all-reduced and detached)."""
    from .tower_code.v1_usertower_train import packed_out

    rank, ws = world()
    device = batch["item_ids"].device
    if index is None:
        index = prepare_step_index(batch, pretrained_vecs, pretrained_lookup)
    else:
        _adopt(index)
    B = index.B
    # tail: the tower's last layer past attention and its output head run only on the rows read
    # here (all of view 1; view 2's "last" row per user, rows T..T+B-1 of `out`)
    pk, out = packed_out(model, batch, pretrained_vecs, pretrained_lookup, packed=index.packed, tail=True)
    # the loss rows of view 1 (valid steps, normalised again: the reference's F.normalize of the
    # already-normalised output) and the "last" rows of both views, gathered by one autograd node
    # whose backward writes a single gradient of `out`
    T = pk.flat.numel()
    last2 = torch.arange(T, T + pk.last_tok.numel(), device=out.device)
    u_loc, z1, z2 = ops.gather_rows_multi(out, [(pk.valid_tok, True), (pk.last_tok, True), (last2, True)])

    # ---- main LogQ loss over all valid steps of the global batch
    n_glob = index.n_glob
    main_sum = None
    if n_glob > 0:
        groups = index.groups
        items_d = ops.gather_rows(item_tower.get_all_embeddings(), groups.uniq, normalize=True, unique=True)
        bias = None
        if cfg.lambda_logq > 0.0:
            bias = log_q_tensor[groups.uniq]
            if cfg.lambda_logq != 1.0:
                bias = bias * cfg.lambda_logq
        main_sum, _ = ops.nce_grouped_sum(u_loc, items_d, bias, groups, tau=temperature, tag="main")

    # ---- DuoRec on the bug-compatible "last" index (count_valid - 1), global B x B
    last_t = index.last_t
    bcounts = [B] * ws
    b_glob = B * ws
    z1_glob = all_gather_rows(z1, bcounts)
    z2_glob = all_gather_rows(z2, bcounts)
    t_glob_last = index.t_glob_last
    un_sum, _ = ops.nce_sum(z1, z2_glob, tau=temperature, flags=ops.NCE_PLAIN, diag_offset=rank * B,
                            tag="duorec")
    sup_sum = cnt_glob = None
    if cfg.lambda_sup > 0:
        sup_sum, sup_cnt = ops.nce_sum(z1, z1_glob, None, last_t, t_glob_last, tau=temperature,
                                       flags=ops.NCE_SUPCON, diag_offset=rank * B, tag="supcon")
        cnt_glob = sup_cnt.detach()
        if ws > 1:
            cnt_glob = all_reduce_sum_(cnt_glob.clone())
    # objective = main / n_glob + lambda_cl * (unsup / b_glob + lambda_sup * sup / max(cnt_glob, 1)),
    # one device launch (ops.loss_combine) instead of ~10 scalar tensor ops and their backward
    objective, logs = ops.loss_combine(main_sum, un_sum, sup_sum, cnt_glob, n_glob, b_glob, cfg.lambda_sup,
                                       cfg.lambda_cl)
    all_reduce_sum_(logs)
    return objective, logs[0], logs[1], logs[2]


def contrastive_step_dp(model, item_tower, log_q_tensor, batch, optimizer, cfg, pretrained_lookup, bucket,
                        max_norm=5.0, index=None):
    """Full data-parallel step: local forward/loss/backward, one gradient all-reduce,
    clip_grad_norm_(5.0) on the summed gradients, AdamW (replicated, identical on all ranks).
    index: the batch's StepIndex prepared ahead (e.g. prepare_step_index_async while the
    previous step runs); built inline if None."""
    ops.zero_grad_(optimizer)
    objective, total, main, cl = contrastive_objective_dp(model, item_tower, log_q_tensor, batch, cfg,
                                                          pretrained_lookup=pretrained_lookup, index=index)
    objective.backward()
    bucket()
    # clip + AdamW in two launches (rsx_clip_adamw); torch's pair for optimizers it does not cover
    if ops.clip_adamw_step(optimizer, ops.module_params(model), max_norm) is None:
        torch.nn.utils.clip_grad_norm_(model.parameters(), max_norm=max_norm)
        optimizer.step()
    return total, main, cl


def merge_topk(scores, idx, k):
    """Top-k of candidate lists [Q, C] by (score desc, index asc): the deterministic merge
    of per-shard results."""
    order = torch.argsort(idx, dim=1, stable=True)
    s1 = torch.gather(scores, 1, order)
    i1 = torch.gather(idx, 1, order)
    o2 = torch.argsort(-s1, dim=1, stable=True)[:, :k]
    return torch.gather(s1, 1, o2), torch.gather(i1, 1, o2)


def retrieve_topk_sharded(queries, item_shard, shard_offset, k, local_topk=None, group=None):
    """Retrieval over an item corpus sharded by row range across ranks:
    each rank takes the top-k of its shard (rsx_retrieve_topk, indices made global with
    shard_offset), the [Q, k] lists are all-gathered, and every rank merges them by
    (score desc, index asc). Shards with fewer than k rows pad with (-inf, -1).
    local_topk(queries, items, k) -> (scores, idx) defaults to ops.retrieve_topk."""
    local_topk = local_topk or ops.retrieve_topk
    kk = min(k, item_shard.shape[0])
    if kk > 0:
        s, i = local_topk(queries, item_shard, kk)
        s = s.to(torch.float32)
        i = torch.where(i >= 0, i + shard_offset, torch.full_like(i, -1))
    else:
        s = queries.new_empty(queries.shape[0], 0)
        i = torch.empty(queries.shape[0], 0, dtype=torch.int64, device=queries.device)
    if kk < k:
        pad = k - kk
        s = torch.cat([s, s.new_full((s.shape[0], pad), float("-inf"))], 1)
        i = torch.cat([i, i.new_full((i.shape[0], pad), -1)], 1)
    i = torch.where(i < 0, torch.full_like(i, torch.iinfo(torch.int64).max), i)
    rank, ws = world()
    if ws > 1:
        ss = [torch.empty_like(s) for _ in range(ws)]
        ii = [torch.empty_like(i) for _ in range(ws)]
        all_gather_into(ss, s.contiguous(), group=group)
        all_gather_into(ii, i.contiguous(), group=group)
        s = torch.cat(ss, 1)
        i = torch.cat(ii, 1)
    s, i = merge_topk(s, i, k)
    i = torch.where(i == torch.iinfo(torch.int64).max, torch.full_like(i, -1), i)
    return s, i
