"""Autograd-aware wrappers over the C-ABI kernels (include/recsys_amd.h).

Every function here launches HIP kernels from librecsys_amd.so on the current torch stream.
There is no CPU path: a non-ROCm tensor raises.
"""
from __future__ import annotations

import ctypes
import os
import weakref

import torch

from . import _native as N

NCE_PLAIN = 0
NCE_MASK_ITEM = 2
NCE_MASK_ITEM_USER = 6
NCE_SUPCON = 9

_NSPLIT_FWD = 8
# partial slots of the grouped forward; the fused forward (rsx_nce_grouped_fwd_grad) accepts 1/2/4/8 and
# runs 4 splits on the leading row blocks, 8 on the tail
_NSPLIT_FWD_GROUPED = int(os.environ.get("RSX_NCE_NSPLIT_FWD", "2"))
if _NSPLIT_FWD_GROUPED not in (1, 2, 4, 8):
    raise ValueError("RSX_NCE_NSPLIT_FWD must be 1, 2, 4 or 8 (the fused forward's supported partial-slot counts)")
_NSPLIT_BWD = 8

# Logit precision of the grouped (live LogQ) loss kernels, include/recsys_amd.h RSX_NCE_*:
# "bf16x3" = hi/lo bf16 split on the bf16 MFMA (max |dot error| ~3e-6 on unit vectors; the
# reference computes these logits in fp16 under AMP), "fp32" = fp32-input MFMA, "f16" = the fused
# forward and the column pass on the fp16 MFMA: logits from an fp16 hi/lo split (tighter than
# bf16x3), gradient products as one fp16 MFMA (the reference's autocast-fp16 arithmetic for them).
NCE_PRECISIONS = {"fp32": 0, "bf16x3": 1, "f16": 2}
_nce_precision = os.environ.get("RSX_NCE_PRECISION", "f16")
if _nce_precision not in NCE_PRECISIONS:
    raise ValueError(f"RSX_NCE_PRECISION must be one of {sorted(NCE_PRECISIONS)}")


def set_nce_precision(mode: str) -> str:
    """Set the grouped-loss precision ("fp32" | "bf16x3" | "f16"); returns the previous mode."""
    global _nce_precision
    if mode not in NCE_PRECISIONS:
        raise ValueError(f"precision must be one of {sorted(NCE_PRECISIONS)}")
    prev, _nce_precision = _nce_precision, mode
    return prev


def nce_precision() -> str:
    return _nce_precision


def next_seed() -> int:
    """Dropout seed from torch's CPU generator (reproducible under torch.manual_seed)."""
    return int(torch.randint(0, 2**62, (1,), dtype=torch.int64).item())


def _c(t):
    return t if t is None or t.is_contiguous() else t.contiguous()


def _tensor_key(ts):
    """Cache key of derived device images: the tensor OBJECTS (held, so their storage cannot be
    recycled under a stale key), their storage pointers and in-place version counters."""
    return tuple((t, t.data_ptr(), t._version) for t in ts)


def _key_eq(a, b) -> bool:
    """Key equality with identity for tensors (== on tensors is elementwise)."""
    if a is None or len(a) != len(b):
        return False
    for x, y in zip(a, b):
        if isinstance(x, tuple):
            if x[0] is not y[0] or x[1:] != y[1:]:
                return False
        elif x != y:
            return False
    return True


# ----------------------------------------------------------------------------------------
# A2: fused sequence embedding (v1_refine_usertower.py:447-459)
def _zeros_group(likes):
    """Zero gradient buffers shaped like each tensor in likes (None -> None), carved out of ONE
    zero-filled allocation (one fill launch instead of one per table); 16-B aligned slices."""
    shapes = [None if t is None else t.shape for t in likes]
    sizes = [0 if t is None else (t.numel() + 3) // 4 * 4 for t in likes]
    total = sum(sizes)
    if total == 0:
        return [None] * len(likes)
    ref = next(t for t in likes if t is not None)
    flat = torch.zeros(total, device=ref.device, dtype=torch.float32)
    out, o = [], 0
    for shp, n, t in zip(shapes, sizes, likes):
        out.append(None if t is None else flat[o:o + t.numel()].view(shp))
        o += n
    return out


class _SeqEmbed(torch.autograd.Function):
    @staticmethod
    def forward(ctx, base, gate, pos, ln_w, ln_b, ids, cfg, tok_pos, *tables):
        eps, p_drop, seed, padding_idx, L, tab0_seg = cfg
        N.ensure_device(base)
        D = base.shape[-1]
        T = base.numel() // D
        base = _c(base)
        ids = [_c(t) for t in ids]
        tables = [_c(t) for t in tables]
        out = torch.empty_like(base)
        mean = torch.empty(T, device=base.device, dtype=torch.float32)
        rstd = torch.empty_like(mean)
        gate = _c(gate)
        with timed("seq_embed_fwd"):
            rc = N.lib().rsx_seq_embed_fwd(
                N.ptr(base), N.ptr_array(ids), N.ptr_array(tables), len(tables), N.ptr(gate), N.ptr(pos),
                N.ptr(tok_pos), N.ptr(ln_w), N.ptr(ln_b), eps, T, L, D, p_drop, seed, N.ptr(out), N.ptr(mean),
                N.ptr(rstd), N.stream())
        N.check(rc, "seq_embed_fwd")
        ctx.save_for_backward(base, gate, pos, ln_w, mean, rstd, tok_pos, *ids, *tables)
        ctx.cfg = (eps, p_drop, seed, padding_idx, len(tables), T, L, D)
        ctx.tab0_seg = tab0_seg
        return out

    @staticmethod
    def backward(ctx, dout):
        eps, p_drop, seed, padding_idx, nt, T, L, D = ctx.cfg
        saved = ctx.saved_tensors
        base, gate, pos, ln_w, mean, rstd, tok_pos = saved[:7]
        ids = list(saved[7:7 + nt])
        tables = list(saved[7 + nt:7 + 2 * nt])
        dout = _c(dout)
        need = ctx.needs_input_grad
        dbase = torch.empty_like(base) if need[0] else None
        dgate, dpos, dlnw, dlnb, *dtabs = _zeros_group(
            [gate if need[1] else None, pos if need[2] else None, ln_w if need[3] else None,
             ln_w if need[4] else None] + [t if need[8 + j] else None for j, t in enumerate(tables)])
        rows = N.i64_array([t.shape[0] for t in tables])
        # table 0 with a prepared sort by id: segmented sums of dx (= dbase) instead of atomics
        seg0 = ctx.tab0_seg if (nt > 0 and dtabs[0] is not None) else None
        if seg0 is not None and dbase is None:
            dbase = torch.empty_like(base)
        kern_tabs = ([None] + dtabs[1:]) if seg0 is not None else dtabs
        nws = N.lib().rsx_seq_embed_bwd_workspace_floats(T, L, D)
        ws = torch.empty(nws, device=base.device, dtype=torch.float32)
        with timed("seq_embed_bwd"):
            rc = N.lib().rsx_seq_embed_bwd(
                N.ptr(base), N.ptr_array(ids), N.ptr_array(tables), rows,
                N.i64_array(padding_idx), nt, N.ptr(gate), N.ptr(pos), N.ptr(tok_pos), N.ptr(ln_w), N.ptr(mean),
                N.ptr(rstd), eps, T, L, D, p_drop, seed, N.ptr(dout), N.ptr(dbase), N.ptr_array(kern_tabs),
                N.ptr(dgate), N.ptr(dpos), N.ptr(dlnw), N.ptr(dlnb), N.ptr(ws), nws, N.stream())
        N.check(rc, "seq_embed_bwd")
        if seg0 is not None:  # chunk partials, then per-id sums of its chunks (both deterministic)
            perm, cb, chunk_ids, ch_off, uniq = seg0
            part = torch.empty(chunk_ids.numel(), D, device=base.device, dtype=torch.float32)
            rc = N.lib().rsx_segment_sum_rows(N.ptr(dbase), D, N.ptr(perm), N.ptr(cb), N.ptr(chunk_ids),
                                              chunk_ids.numel(), D, None, -1, N.ptr(part), D, 0, N.stream())
            N.check(rc, "segment_sum_rows(chunks)")
            rc = N.lib().rsx_segment_sum_rows(N.ptr(part), D, N.ptr(chunk_ids), N.ptr(ch_off), N.ptr(uniq),
                                              uniq.numel(), D, N.ptr(gate), padding_idx[0], N.ptr(dtabs[0]),
                                              dtabs[0].stride(0), 1, N.stream())
            N.check(rc, "segment_sum_rows(ids)")
        if not need[0]:
            dbase = None
        return (dbase, dgate, dpos, dlnw, dlnb, None, None, None, *dtabs)


_SEG_CHUNK = 64


def sort_segments(ids):
    """Two-level plan for the sorted segmented sums of table 0's gradient (seq_embed tab0_seg):
    ids[perm] sorted (stable); the sorted tokens are cut into chunks of <= 64 tokens that never
    straddle two ids (chunk c = [cb[c], cb[c+1])), so a Zipf-hot id's thousands of tokens are
    summed by many chunks in parallel; segment u (id uniq[u]) owns chunks [ch_off[u],
    ch_off[u+1]). Its size queries synchronise the host (build it ahead, e.g. in
    dist.prepare_step_index_async). Returns (perm, cb, chunk_ids, ch_off, uniq)."""
    ids = ids.reshape(-1)
    dev = ids.device
    srt, perm = torch.sort(ids, stable=True)
    uniq, cnt = torch.unique_consecutive(srt, return_counts=True)
    seg_off = torch.zeros(uniq.numel() + 1, device=dev, dtype=torch.int64)
    seg_off[1:] = torch.cumsum(cnt, 0)
    nch = (cnt + _SEG_CHUNK - 1) // _SEG_CHUNK
    ch_off = torch.zeros(uniq.numel() + 1, device=dev, dtype=torch.int64)
    ch_off[1:] = torch.cumsum(nch, 0)
    total = int(ch_off[-1])
    ch_seg = torch.repeat_interleave(torch.arange(uniq.numel(), device=dev), nch, output_size=total)
    k = torch.arange(total, device=dev)
    cb = torch.empty(total + 1, device=dev, dtype=torch.int64)
    cb[:-1] = seg_off[ch_seg] + _SEG_CHUNK * (k - ch_off[ch_seg])
    cb[-1] = ids.numel()
    return perm, cb, k, ch_off, uniq


def seq_embed(base, ids, tables, gate, pos, ln_w, ln_b, eps=1e-5, p_drop=0.0, padding_idx=None, tok_pos=None,
              tab0_seg=None):
    """x = base + sum_j tables[j][ids[j]] * gate[j] + pos[l] ; LayerNorm ; dropout.

    Dense: base [B, L, D], ids [B, L], pos [>= L, D] (position = token % L).
    Packed: base [T, D], ids [T], tok_pos [T] int64 positions, pos [L, D].
    gate [ntab]; ln_w/ln_b [D]. padding_idx: per-table row excluded from the table gradient
    (nn.Embedding semantics). tab0_seg: sort_segments(ids[0]) — table 0's gradient then comes
    from rsx_segment_sum_rows (deterministic, no atomics) instead of the kernel's scatter-add.
    """
    if padding_idx is None:
        padding_idx = [-1] * len(tables)
    padding_idx = [(-1 if p is None else int(p)) for p in padding_idx]
    seed = next_seed() if p_drop > 0 else 0
    if tok_pos is None:
        L = base.shape[1]
        pos = pos[:L]
    else:
        L = pos.shape[0]
        tok_pos = _c(tok_pos)
    cfg = (float(eps), float(p_drop), seed, padding_idx, int(L), tab0_seg)
    return _SeqEmbed.apply(base, gate, pos, ln_w, ln_b, list(ids), cfg, tok_pos, *tables)


# ----------------------------------------------------------------------------------------
# A3 / A9: masked MHA core
# "bf16x3" (default): head dim 32 runs mha_fwd_x3_k / mha_bwd_x3_k (split-bf16 MFMA, ~2^-17
# relative error per product); other head dims and "fp32" run the fp32 kernels.
MHA_PRECISIONS = ("fp32", "bf16x3")
_mha_precision = os.environ.get("RSX_MHA_PRECISION", "bf16x3")
assert _mha_precision in MHA_PRECISIONS, _mha_precision


def set_mha_precision(p: str) -> None:
    global _mha_precision
    assert p in MHA_PRECISIONS, p
    _mha_precision = p


def mha_precision() -> str:
    return _mha_precision


def _mha_x3(Dh):
    return _mha_precision == "bf16x3" and Dh == 32


def _mha_x3_fwd(Dh):  # the bf16x3 forward also covers head dim 64 (BERT inference; no x3 backward)
    return _mha_precision == "bf16x3" and Dh in (32, 64)


class _MHA(torch.autograd.Function):
    @staticmethod
    def forward(ctx, qkv, key_pad, seg_off, H, causal, p_drop, seed, max_len=None):
        N.ensure_device(qkv)
        qkv = _c(qkv)
        D3 = qkv.shape[-1]
        T = qkv.numel() // D3
        D = D3 // 3
        Dh = D // H
        if seg_off is None:
            B, L = qkv.shape[0], qkv.shape[1]
        else:  # packed: L bounds the segment lengths (the head-dim-64 backward sizes its LDS by it)
            B, L = seg_off.numel() - 1, int(max_len) if max_len else 64
        out = torch.empty(qkv.shape[:-1] + (D,), device=qkv.device, dtype=torch.float32)
        lse = torch.empty(T, H, device=qkv.device, dtype=torch.float32)
        kp = None
        if key_pad is not None:
            kp = _c(key_pad.to(torch.uint8)) if key_pad.dtype != torch.uint8 else _c(key_pad)
        fn = N.lib().rsx_mha_fwd_x3 if _mha_x3_fwd(Dh) else N.lib().rsx_mha_fwd
        rc = fn(N.ptr(qkv), N.ptr(kp), N.ptr(seg_off), B, L, H, Dh, int(causal), p_drop, seed, N.ptr(out), N.ptr(lse),
                N.stream())
        N.check(rc, "mha_fwd")
        ctx.save_for_backward(qkv, kp, seg_off, out, lse)
        ctx.cfg = (B, L, H, Dh, int(causal), p_drop, seed)
        return out

    @staticmethod
    def backward(ctx, dout):
        B, L, H, Dh, causal, p_drop, seed = ctx.cfg
        qkv, kp, seg_off, out, lse = ctx.saved_tensors
        dout = _c(dout)
        dqkv = torch.empty_like(qkv)
        fn = N.lib().rsx_mha_bwd_x3 if _mha_x3(Dh) else N.lib().rsx_mha_bwd
        rc = fn(N.ptr(qkv), N.ptr(kp), N.ptr(seg_off), N.ptr(out), N.ptr(lse), N.ptr(dout), B, L, H, Dh, causal,
                p_drop, seed, N.ptr(dqkv), N.stream())
        N.check(rc, "mha_bwd")
        return dqkv, None, None, None, None, None, None, None


class _QKVMHA(torch.autograd.Function):
    """mha(F.linear(x, w, b)) with the projection fused into the attention forward
    (rsx_mha_qkv_fwd_x3: head dim 32, D = 128, bf16x3). The kernel still writes qkv, which the
    backward uses exactly as _MHA + _TokLinear do: dqkv from rsx_mha_bwd_x3, then dx on the
    bf16x3 GEMM and (dw, db) from the split-K weight-gradient kernel."""

    @staticmethod
    def forward(ctx, x, w, b, key_pad, seg_off, H, causal, p_drop, seed):
        N.ensure_device(x)
        x = _c(x)
        w = _c(w)
        D = x.shape[-1]
        T = x.numel() // D
        if seg_off is None:
            B, L = x.shape[0], x.shape[1]
        else:
            B, L = seg_off.numel() - 1, 64
        qkv = torch.empty(x.shape[:-1] + (3 * D,), device=x.device, dtype=torch.float32)
        out = torch.empty_like(x)
        lse = torch.empty(T, H, device=x.device, dtype=torch.float32)
        kp = None
        if key_pad is not None:
            kp = _c(key_pad.to(torch.uint8)) if key_pad.dtype != torch.uint8 else _c(key_pad)
        with timed("qkv_mha_fwd"):
            rc = N.lib().rsx_mha_qkv_fwd_x3(N.ptr(x), N.ptr(w), N.ptr(None if b is None else _c(b)), N.ptr(kp),
                                            N.ptr(seg_off), B, L, H, int(causal), p_drop, seed, N.ptr(qkv),
                                            N.ptr(out), N.ptr(lse), N.stream())
        N.check(rc, "mha_qkv_fwd_x3")
        ctx.save_for_backward(x, w, qkv, kp, seg_off, out, lse)
        ctx.cfg = (B, L, H, int(causal), p_drop, seed, b is not None)
        return out

    @staticmethod
    def backward(ctx, dout):
        B, L, H, causal, p_drop, seed, has_bias = ctx.cfg
        x, w, qkv, kp, seg_off, out, lse = ctx.saved_tensors
        dout = _c(dout)
        dqkv = torch.empty_like(qkv)
        rc = N.lib().rsx_mha_bwd_x3(N.ptr(qkv), N.ptr(kp), N.ptr(seg_off), N.ptr(out), N.ptr(lse), N.ptr(dout), B, L,
                                    H, 32, causal, p_drop, seed, N.ptr(dqkv), N.stream())
        N.check(rc, "mha_bwd")
        D = x.shape[-1]
        dq2 = dqkv.reshape(-1, 3 * D)
        dx = _dx(dq2, w).reshape(x.shape) if ctx.needs_input_grad[0] else None
        dw = db = None
        if ctx.needs_input_grad[1] or (has_bias and ctx.needs_input_grad[2]):
            dw, db = linear_wgrad(dq2, x.reshape(-1, D), w.shape, has_bias and ctx.needs_input_grad[2])
        return dx, dw, db, None, None, None, None, None, None


# RSX_QKV_FUSED=1 opts into the fused projection + attention kernel. Off by default:
# measured 0.879 ms vs 0.358 ms for linear_tok + mha at the step shape (the fused
# kernel recomputes the K/V projection per query block and runs at 272 VGPRs).
_QKV_FUSED = os.environ.get("RSX_QKV_FUSED", "0") == "1"


def qkv_mha(x, w, b, key_pad, num_heads, causal, p_drop=0.0, seg_off=None):
    """mha(linear(x, w, b), ...): the fused projection + attention kernel when it applies
    (bf16x3 mode, 4 heads of 32, dense or packed), otherwise linear_tok then mha."""
    D = x.shape[-1]
    if (_QKV_FUSED and _mha_precision == "bf16x3" and _gemm_precision == "bf16x3" and D == 128
            and int(num_heads) == 4 and tuple(w.shape) == (3 * D, D) and x.is_cuda):
        seed = next_seed() if p_drop > 0 else 0
        if seg_off is not None:
            seg_off = _c(seg_off.to(torch.int32))
        return _QKVMHA.apply(x, w, b, key_pad, seg_off, 4, bool(causal), float(p_drop), seed)
    return mha(linear_tok(x, w, b), key_pad, num_heads, causal, p_drop, seg_off)


def mha(qkv, key_pad, num_heads, causal, p_drop=0.0, seg_off=None, max_len=None):
    """Dense: qkv [B, L, 3D], key_pad [B, L]. Packed: qkv [T, 3D], key_pad [T], seg_off [B+1] int32;
    max_len (packed, optional) = an upper bound of the segment lengths (<= 64)."""
    seed = next_seed() if p_drop > 0 else 0
    if seg_off is not None:
        seg_off = _c(seg_off.to(torch.int32))
    return _MHA.apply(qkv, key_pad, seg_off, int(num_heads), bool(causal), float(p_drop), seed, max_len)


# ----------------------------------------------------------------------------------------
# Row gather (+ optional F.normalize) with scatter backward
class _GatherRows(torch.autograd.Function):
    @staticmethod
    def forward(ctx, src, idx, normalize, eps, unique, skip_idx):
        N.ensure_device(src)
        D = src.shape[-1]
        src2 = src.reshape(-1, D)
        if src2.stride(1) != 1 or src2.stride(0) % 4 != 0 or src2.data_ptr() % 16 != 0:
            src2 = src2.contiguous()
        n = idx.numel() if idx is not None else src2.shape[0]
        idx_c = _c(idx) if idx is not None else None
        out = torch.empty(n, D, device=src.device, dtype=torch.float32)
        nrm = torch.empty(n, device=src.device, dtype=torch.float32) if normalize else None
        rc = N.lib().rsx_gather_rows(N.ptr(src2), src2.stride(0), N.ptr(idx_c), n, D, int(normalize), eps,
                                     N.ptr(out), N.ptr(nrm), N.stream())
        N.check(rc, "gather_rows")
        ctx.src_shape = src.shape
        ctx.cfg = (normalize, eps, unique, skip_idx, n, D)
        saved = [t for t in (idx_c, out if normalize else None, nrm) if t is not None]
        ctx.has_idx = idx_c is not None
        ctx.save_for_backward(*saved)
        return out

    @staticmethod
    def backward(ctx, dy):
        normalize, eps, unique, skip_idx, n, D = ctx.cfg
        saved = list(ctx.saved_tensors)
        idx = saved.pop(0) if ctx.has_idx else None
        y = nrm = None
        if normalize:
            y, nrm = saved
        dy = _c(dy)
        rows = 1
        for s in ctx.src_shape[:-1]:
            rows *= s
        if idx is None:
            dsrc = torch.empty(rows, D, device=dy.device, dtype=torch.float32)
            mode = 0
        else:
            dsrc = torch.zeros(rows, D, device=dy.device, dtype=torch.float32)
            mode = 1 if unique else 2
        rc = N.lib().rsx_scatter_rows(N.ptr(dy), N.ptr(y), N.ptr(nrm), N.ptr(idx), n, D, int(normalize), eps, mode,
                                      skip_idx, N.ptr(dsrc), D, N.stream())
        N.check(rc, "scatter_rows")
        return dsrc.view(ctx.src_shape), None, None, None, None, None


def gather_rows(src, idx=None, normalize=False, eps=1e-12, unique=False, skip_idx=-1):
    """out[r] = src.view(-1, D)[idx[r]] (idx None => all rows), optionally L2-normalised. The kernel
    reads fp32 rows: another floating dtype is cast first (autograd-aware), anything else refused."""
    if src.dtype != torch.float32:
        if not src.is_floating_point():
            raise TypeError(f"gather_rows: floating-point rows expected, got {src.dtype}")
        src = src.float()
    return _GatherRows.apply(src, idx, bool(normalize), float(eps), bool(unique), int(skip_idx))


class _GatherRowsMulti(torch.autograd.Function):
    """Several row gathers of one source (each index list duplicate-free), with ONE zero-filled
    source gradient that every gather's backward accumulates into in turn (non-atomic
    read-add-write, scatter mode 1): the autograd form of k gathers of slices of one tensor
    costs k zero-filled gradients, the slice gradients and their sums."""

    @staticmethod
    def forward(ctx, src, norms, eps, *idxs):
        N.ensure_device(src)
        src2 = _c(src)
        D = src2.shape[-1]
        outs, saved = [], []
        for idx, nz in zip(idxs, norms):
            idx = _c(idx)
            n = idx.numel()
            out = torch.empty(n, D, device=src.device, dtype=torch.float32)
            nrm = torch.empty(n, device=src.device, dtype=torch.float32) if nz else None
            rc = N.lib().rsx_gather_rows(N.ptr(src2), src2.stride(0), N.ptr(idx), n, D, int(nz), eps, N.ptr(out),
                                         N.ptr(nrm), N.stream())
            N.check(rc, "gather_rows")
            outs.append(out)
            saved += [idx, out if nz else idx, nrm if nz else idx]
        ctx.cfg = (tuple(norms), eps, src2.shape)
        ctx.save_for_backward(*saved)
        return tuple(outs)

    @staticmethod
    def backward(ctx, *dys):
        norms, eps, shape = ctx.cfg
        saved = ctx.saved_tensors
        D = shape[-1]
        dsrc = torch.zeros(shape, device=saved[0].device, dtype=torch.float32)
        for k, (dy, nz) in enumerate(zip(dys, norms)):
            if dy is None:
                continue
            idx, y, nrm = saved[3 * k], saved[3 * k + 1], saved[3 * k + 2]
            dy = _c(dy)
            rc = N.lib().rsx_scatter_rows(N.ptr(dy), N.ptr(y if nz else None), N.ptr(nrm if nz else None), N.ptr(idx),
                                          idx.numel(), D, int(nz), eps, 1, -1, N.ptr(dsrc), D, N.stream())
            N.check(rc, "scatter_rows")
        return (dsrc, None, None) + (None,) * len(dys)


def gather_rows_multi(src, specs, eps=1e-12):
    """[gather_rows(src, idx, normalize=nz, unique=True) for idx, nz in specs] as one autograd
    node (one source gradient buffer; each idx must be duplicate-free)."""
    idxs = [i for i, _ in specs]
    norms = [bool(nz) for _, nz in specs]
    return list(_GatherRowsMulti.apply(src, norms, float(eps), *idxs))


def l2_normalize(x, eps=1e-12):
    """F.normalize(x, p=2, dim=-1) on the last dim."""
    shape = x.shape
    return gather_rows(x, None, normalize=True, eps=eps).view(shape)


# ----------------------------------------------------------------------------------------
# A6 / A7 / A12: fused contrastive cross-entropy
class _NCE(torch.autograd.Function):
    """Returns (sum of row losses over valid rows, number of valid rows). bf16x3 precision
    (default) runs rsx_nce_fwd_x3 / rsx_nce_bwd_x3 (split counts chosen by the library), fp32
    the fp32-MFMA rsx_nce_fwd / rsx_nce_bwd."""

    @staticmethod
    def forward(ctx, A, B, bias, k1a, k1b, k2a, k2b, tau, flags, diag_offset, tag):
        N.ensure_device(A)
        A = _c(A)
        B = _c(B)
        n, m = A.shape[0], B.shape[0]
        x3 = _nce_precision != "fp32"  # "f16" only changes the grouped kernels
        nws = (N.lib().rsx_nce_x3_workspace_floats(n, m) if x3
               else N.lib().rsx_nce_workspace_floats(n, m, _NSPLIT_FWD, _NSPLIT_BWD))
        ws = torch.empty(nws, device=A.device, dtype=torch.float32)
        out2 = torch.empty(2, device=A.device, dtype=torch.float32)
        keys = [_c(k) for k in (k1a, k1b, k2a, k2b)]
        with timed(f"{tag}/nce_fwd"):
            if x3:
                rc = N.lib().rsx_nce_fwd_x3(N.ptr(A), N.ptr(B), N.ptr(bias), *[N.ptr(k) for k in keys], n, m,
                                            A.stride(0), B.stride(0), diag_offset, tau, flags, N.ptr(ws), N.ptr(out2),
                                            N.stream())
            else:
                rc = N.lib().rsx_nce_fwd(N.ptr(A), N.ptr(B), N.ptr(bias), *[N.ptr(k) for k in keys], n, m,
                                         A.stride(0), B.stride(0), diag_offset, tau, flags, _NSPLIT_FWD, N.ptr(ws),
                                         N.ptr(out2), N.stream())
        N.check(rc, "nce_fwd")
        ctx.save_for_backward(A, B, bias, *keys, ws)
        ctx.cfg = (n, m, tau, flags, diag_offset, tag, x3)
        cnt = out2[1]
        ctx.mark_non_differentiable(cnt)
        return out2[0], cnt

    @staticmethod
    def backward(ctx, g, _gcnt):
        A, B, bias, k1a, k1b, k2a, k2b, ws = ctx.saved_tensors
        n, m, tau, flags, off, tag, x3 = ctx.cfg
        g = _c(g.reshape(1).to(torch.float32))
        head = (N.ptr(A), N.ptr(B), N.ptr(bias), N.ptr(k1a), N.ptr(k1b), N.ptr(k2a), N.ptr(k2b), n, m, A.stride(0),
                B.stride(0), off, tau, flags)
        if x3:
            fn, args = N.lib().rsx_nce_bwd_x3, head + (N.ptr(g), N.ptr(ws))
        else:
            fn, args = N.lib().rsx_nce_bwd, head + (_NSPLIT_FWD, _NSPLIT_BWD, N.ptr(g), N.ptr(ws))
        dA = dB = None
        if ctx.needs_input_grad[0]:
            dA = torch.empty_like(A)
            with timed(f"{tag}/nce_bwd_rows"):
                rc = fn(*args, N.ptr(dA), None, 0, N.stream())
            N.check(rc, "nce_bwd(rows)")
        if ctx.needs_input_grad[1]:
            dB = torch.empty_like(B)
            with timed(f"{tag}/nce_bwd_cols"):
                rc = fn(*args, None, N.ptr(dB), 0, N.stream())
            N.check(rc, "nce_bwd(cols)")
        return dA, dB, None, None, None, None, None, None, None, None, None


def _i32(t):
    return None if t is None else t.to(torch.int32)


def nce_sum(A, B, bias=None, k1a=None, k1b=None, k2a=None, k2b=None, tau=0.1, flags=NCE_PLAIN, diag_offset=0,
            tag="nce"):
    """(sum of row losses, valid-row count) of S = A B^T / tau - bias; row i's label column
    is i + diag_offset (see include/recsys_amd.h)."""
    if bias is not None:
        bias = _c(bias.to(torch.float32))
    return _NCE.apply(A, B, bias, _i32(k1a), _i32(k1b), _i32(k2a), _i32(k2b), float(tau), int(flags),
                      int(diag_offset), str(tag))


def nce_loss(A, B, bias=None, k1a=None, k1b=None, k2a=None, k2b=None, tau=0.1, flags=NCE_PLAIN, tag="nce"):
    """Mean InfoNCE over valid rows (0 if none), the reference's F.cross_entropy mean."""
    total, cnt = nce_sum(A, B, bias, k1a, k1b, k2a, k2b, tau, flags, tag=tag)
    return total / cnt.clamp(min=1.0)


class _NCEEmphasis(torch.autograd.Function):
    """(sum of row losses, N) of full_batch_hard_emphasis_loss's cross-entropy (v1_refine_usertower.py
    :762-822): S = A B^T / tau - bias, same-key columns off the diagonal excluded (flags MASK_K1), and
    +margin on each row's mined columns top [N, K] -- the dense flags-2 InfoNCE pass plus the O(N K)
    rsx_nce_emphasis_fwd / _bwd correction; no N x N tensor."""

    @staticmethod
    def forward(ctx, A, B, bias, k1, top, tau, margin, tag):
        N.ensure_device(A)
        A = _c(A)
        B = _c(B)
        n, m = A.shape[0], B.shape[0]
        K = top.shape[1] if top.dim() == 2 else 0
        top = _c(top.to(torch.int64))
        x3 = _nce_precision != "fp32"
        prec = 1 if x3 else 0
        nws = (N.lib().rsx_nce_x3_workspace_floats(n, m) if x3
               else N.lib().rsx_nce_workspace_floats(n, m, _NSPLIT_FWD, _NSPLIT_BWD))
        ws = torch.empty(nws, device=A.device, dtype=torch.float32)
        out2 = torch.empty(2, device=A.device, dtype=torch.float32)
        flags = NCE_MASK_ITEM
        with timed(f"{tag}/nce_fwd"):
            if x3:
                rc = N.lib().rsx_nce_fwd_x3(N.ptr(A), N.ptr(B), N.ptr(bias), N.ptr(k1), N.ptr(k1), None, None, n, m,
                                            A.stride(0), B.stride(0), 0, tau, flags, N.ptr(ws), N.ptr(out2), N.stream())
            else:
                rc = N.lib().rsx_nce_fwd(N.ptr(A), N.ptr(B), N.ptr(bias), N.ptr(k1), N.ptr(k1), None, None, n, m,
                                         A.stride(0), B.stride(0), 0, tau, flags, _NSPLIT_FWD, N.ptr(ws), N.ptr(out2),
                                         N.stream())
            N.check(rc, "nce_fwd")
            rc = N.lib().rsx_nce_emphasis_fwd(N.ptr(A), N.ptr(B), N.ptr(bias), N.ptr(k1), N.ptr(k1), N.ptr(top), n, m,
                                              K, A.stride(0), B.stride(0), 0, tau, margin, prec, _NSPLIT_FWD,
                                              N.ptr(ws), N.ptr(out2), N.stream())
            N.check(rc, "nce_emphasis_fwd")
        # the mined entries in column order (stable: a fixed summation order per column) for the
        # backward's atomic-free dB pass
        flat = top.reshape(-1)
        key = torch.where((flat >= 0) & (flat < m), flat, torch.full_like(flat, m))
        sk, col_ent = torch.sort(key, stable=True)
        col_ptr = torch.searchsorted(sk, torch.arange(m + 1, device=A.device, dtype=sk.dtype))
        ctx.save_for_backward(A, B, bias, k1, top, ws, _c(col_ptr), _c(col_ent))
        ctx.cfg = (n, m, K, tau, margin, tag, x3)
        cnt = out2[1]
        ctx.mark_non_differentiable(cnt)
        return out2[0], cnt

    @staticmethod
    def backward(ctx, g, _gcnt):
        A, B, bias, k1, top, ws, col_ptr, col_ent = ctx.saved_tensors
        n, m, K, tau, margin, tag, x3 = ctx.cfg
        g = _c(g.reshape(1).to(torch.float32))
        head = (N.ptr(A), N.ptr(B), N.ptr(bias), N.ptr(k1), N.ptr(k1), None, None, n, m, A.stride(0), B.stride(0), 0,
                tau, NCE_MASK_ITEM)
        if x3:
            fn, args = N.lib().rsx_nce_bwd_x3, head + (N.ptr(g), N.ptr(ws))
        else:
            fn, args = N.lib().rsx_nce_bwd, head + (_NSPLIT_FWD, _NSPLIT_BWD, N.ptr(g), N.ptr(ws))
        dA = torch.empty_like(A) if ctx.needs_input_grad[0] else None
        dB = torch.empty_like(B) if ctx.needs_input_grad[1] else None
        with timed(f"{tag}/nce_bwd"):
            if dA is not None:
                N.check(fn(*args, N.ptr(dA), None, 0, N.stream()), "nce_bwd(rows)")
            if dB is not None:
                N.check(fn(*args, None, N.ptr(dB), 0, N.stream()), "nce_bwd(cols)")
            if dA is not None or dB is not None:
                cbuf = torch.empty(n * K, device=A.device, dtype=torch.float32) if dB is not None else None
                rc = N.lib().rsx_nce_emphasis_bwd_csr(N.ptr(A), N.ptr(B), N.ptr(bias), N.ptr(k1), N.ptr(k1),
                                                      N.ptr(top), n, m, K, A.stride(0), B.stride(0), 0, tau, margin,
                                                      1 if x3 else 0, _NSPLIT_FWD, N.ptr(col_ptr), N.ptr(col_ent),
                                                      N.ptr(cbuf), N.ptr(g), N.ptr(ws), N.ptr(dA), N.ptr(dB),
                                                      N.stream())
                N.check(rc, "nce_emphasis_bwd")
        return dA, dB, None, None, None, None, None, None


def nce_emphasis_loss(A, B, keys, top, margin, bias=None, tau=0.1, tag="hard_emphasis"):
    """Mean over the N rows of CE(A B^T / tau - bias + margin on each row's mined columns top [N, K],
    same-key columns off the diagonal at -inf; label = diagonal) -- full_batch_hard_emphasis_loss's
    objective (v1_refine_usertower.py:546-554) without its N x N tensors. margin is in logit units
    (the reference's hard_margin / temperature). A [N, 128], B [N, 128], keys [N] int."""
    if A.shape[0] != B.shape[0]:
        raise ValueError("nce_emphasis_loss: A and B must have the same number of rows (label = diagonal)")
    if bias is not None:
        bias = _c(bias.to(torch.float32))
    total, cnt = _NCEEmphasis.apply(A, B, bias, _c(keys.to(torch.int32)), top, float(tau), float(margin), str(tag))
    return total / cnt.clamp(min=1.0)


# ----------------------------------------------------------------------------------------
# Grouped form of the live LogQ loss (distinct targets as columns, exact multiplicities)
class TargetGroups:
    """Index structures for rsx_nce_grouped_*: built on the GPU with a few sorts.

    t_rows/u_rows: this process's rows (flat order; rows of one user are contiguous and user
    ids are non-decreasing). t_cols: every column's target (all ranks' rows; defaults to
    t_rows). The distinct targets of t_cols are the grouped columns."""

    def __init__(self, t_rows, u_rows, t_cols=None):
        t_cols = t_rows if t_cols is None else t_cols
        dev = t_rows.device
        self.uniq, col_cnt = torch.unique(t_cols, sorted=True, return_counts=True)
        D = self.uniq.numel()
        self.colcnt = col_cnt.to(torch.float32)
        inv = torch.searchsorted(self.uniq, t_rows)
        self.row_col = inv.to(torch.int32)
        n = t_rows.numel()
        # rows of each user: [start, end) in flat order
        users, ucnt = torch.unique_consecutive(u_rows, return_counts=True)
        ends = torch.cumsum(ucnt, 0)
        starts = ends - ucnt
        self.row_beg = torch.repeat_interleave(starts, ucnt).to(torch.int32)
        self.row_end = torch.repeat_interleave(ends, ucnt).to(torch.int32)
        # per-row exception list = the user's own targets, sorted within each user segment
        seg = torch.repeat_interleave(torch.arange(users.numel(), device=dev), ucnt)
        key = seg * D + inv
        self.exc_cols = (torch.sort(key).values % D).to(torch.int32)
        # per-column list of (user row range, multiplicity), sorted by column then user
        key2 = inv * users.numel() + seg
        k2, kn = torch.unique_consecutive(torch.sort(key2).values, return_counts=True)
        pd = torch.div(k2, users.numel(), rounding_mode="floor")
        pseg = k2 % users.numel()
        self.exc_s = starts[pseg].to(torch.int32)
        self.exc_e = ends[pseg].to(torch.int32)
        self.exc_n = kn.to(torch.int32)
        ar = torch.arange(D, device=dev)
        self.col_beg = torch.searchsorted(pd, ar).to(torch.int32)
        self.col_end = torch.searchsorted(pd, ar, right=True).to(torch.int32)
        self.n_rows = n
        self.n_cols = D

    @classmethod
    def from_arrays(cls, uniq, colcnt, row_col, row_beg, row_end, exc_cols, exc_s, exc_e, exc_n, col_beg, col_end,
                    n_rows):
        """The same structure from prepared arrays (rsx_step_index_fill, dist.py)."""
        g = cls.__new__(cls)
        g.uniq, g.colcnt, g.row_col, g.row_beg, g.row_end, g.exc_cols = uniq, colcnt, row_col, row_beg, row_end, exc_cols
        g.exc_s, g.exc_e, g.exc_n, g.col_beg, g.col_end = exc_s, exc_e, exc_n, col_beg, col_end
        g.n_rows, g.n_cols = int(n_rows), uniq.numel()
        return g


# bf16x3 + the rows need a gradient: the forward also produces the row gradient (one sweep of
# S instead of two; rsx_nce_grouped_fwd_grad). RSX_NCE_FUSED_ROWGRAD=0 restores the separate
# backward row pass.
_NCE_FUSED_ROWGRAD = os.environ.get("RSX_NCE_FUSED_ROWGRAD", "1") != "0"


class _NCEGrouped(torch.autograd.Function):
    @staticmethod
    def forward(ctx, A, B, bias, grp, tau, tag, prec):
        N.ensure_device(A)
        A = _c(A)
        B = _c(B)
        n, d = A.shape[0], B.shape[0]
        nws = N.lib().rsx_nce_grouped_workspace_floats(n, d, _NSPLIT_FWD_GROUPED, _NSPLIT_BWD, prec)
        ws = torch.empty(nws, device=A.device, dtype=torch.float32)
        out2 = torch.empty(2, device=A.device, dtype=torch.float32)
        fused = _NCE_FUSED_ROWGRAD and prec != NCE_PRECISIONS["fp32"] and ctx.needs_input_grad[0]
        ga = None
        with timed(f"{tag}/nce_fwd"):
            if fused:
                ga = torch.empty(n, 128, device=A.device, dtype=torch.float32)
                rc = N.lib().rsx_nce_grouped_fwd_grad(
                    N.ptr(A), N.ptr(B), N.ptr(bias), N.ptr(grp.colcnt), N.ptr(grp.row_col), N.ptr(grp.row_beg),
                    N.ptr(grp.row_end), N.ptr(grp.exc_cols), n, d, A.stride(0), B.stride(0), tau, prec,
                    _NSPLIT_FWD_GROUPED, N.ptr(ws), N.ptr(out2), N.ptr(ga), N.stream())
            else:
                rc = N.lib().rsx_nce_grouped_fwd(
                    N.ptr(A), N.ptr(B), N.ptr(bias), N.ptr(grp.colcnt), N.ptr(grp.row_col), N.ptr(grp.row_beg),
                    N.ptr(grp.row_end), N.ptr(grp.exc_cols), n, d, A.stride(0), B.stride(0), tau, prec,
                    _NSPLIT_FWD_GROUPED, N.ptr(ws), N.ptr(out2), N.stream())
        N.check(rc, "nce_grouped_fwd")
        ctx.save_for_backward(A, B, bias, ws, ga)
        ctx.grp = grp
        ctx.cfg = (n, d, tau, tag, prec)
        cnt = out2[1]
        ctx.mark_non_differentiable(cnt)
        return out2[0], cnt

    @staticmethod
    def backward(ctx, g, _gcnt):
        A, B, bias, ws, ga = ctx.saved_tensors
        grp = ctx.grp
        n, d, tau, tag, prec = ctx.cfg
        g = _c(g.reshape(1).to(torch.float32))
        args = (N.ptr(A), N.ptr(B), N.ptr(bias), N.ptr(grp.colcnt), N.ptr(grp.row_col), N.ptr(grp.row_beg),
                N.ptr(grp.row_end), N.ptr(grp.exc_cols), N.ptr(grp.col_beg), N.ptr(grp.col_end), N.ptr(grp.exc_s),
                N.ptr(grp.exc_e), N.ptr(grp.exc_n), n, d, A.stride(0), B.stride(0), tau, prec, _NSPLIT_FWD_GROUPED,
                _NSPLIT_BWD,
                N.ptr(g), N.ptr(ws))
        dA = dB = None
        if ctx.needs_input_grad[0]:
            if ga is not None:  # the forward's row gradient, per unit upstream gradient
                dA = ga * g
            else:
                dA = torch.empty_like(A)
                with timed(f"{tag}/nce_bwd_rows"):
                    rc = N.lib().rsx_nce_grouped_bwd(*args, N.ptr(dA), None, 0, N.stream())
                N.check(rc, "nce_grouped_bwd(rows)")
        if ctx.needs_input_grad[1]:
            dB = torch.empty_like(B)
            with timed(f"{tag}/nce_bwd_cols"):
                rc = N.lib().rsx_nce_grouped_bwd(*args, None, N.ptr(dB), 0, N.stream())
            N.check(rc, "nce_grouped_bwd(cols)")
        return dA, dB, None, None, None, None, None


def nce_grouped_sum(A, B_distinct, bias, groups: TargetGroups, tau=0.1, tag="nce", precision=None):
    """(sum of row losses, N) of the live LogQ loss with same-item / same-user masking, with
    the columns given as the distinct targets (B_distinct[d] = normalised item groups.uniq[d]).
    precision: "fp32" | "bf16x3" | "f16" | None (= set_nce_precision / RSX_NCE_PRECISION)."""
    if bias is not None:
        bias = _c(bias.to(torch.float32))
    prec = NCE_PRECISIONS[precision or _nce_precision]
    return _NCEGrouped.apply(A, B_distinct, bias, groups, float(tau), str(tag), prec)


class _LossCombine(torch.autograd.Function):
    """total = s_main / n + lambda_cl * (s_un / b + lambda_sup * s_sup / max(cnt, 1)) on the device
    (rsx_loss_combine), with (total, main, cl) also returned detached for logging."""

    @staticmethod
    def forward(ctx, s_main, s_un, s_sup, cnt, consts):
        inv_n, inv_b, lsup, lcl = consts
        total = torch.empty((), device=s_un.device, dtype=torch.float32)
        logs = torch.empty(3, device=s_un.device, dtype=torch.float32)
        rc = N.lib().rsx_loss_combine(N.ptr(s_main), N.ptr(s_un), N.ptr(s_sup), N.ptr(cnt), inv_n, inv_b, lsup, lcl,
                                      N.ptr(total), N.ptr(logs), N.stream())
        N.check(rc, "loss_combine")
        ctx.consts = consts
        ctx.has = (s_main is not None, s_sup is not None)
        ctx.save_for_backward(cnt)
        ctx.mark_non_differentiable(logs)
        return total, logs

    @staticmethod
    def backward(ctx, g, _glogs):
        (cnt,) = ctx.saved_tensors
        inv_n, inv_b, lsup, lcl = ctx.consts
        g3 = torch.empty(3, device=g.device, dtype=torch.float32)
        rc = N.lib().rsx_loss_combine_bwd(N.ptr(_c(g.reshape(1))), N.ptr(cnt), inv_n, inv_b, lsup, lcl, N.ptr(g3),
                                          N.stream())
        N.check(rc, "loss_combine_bwd")
        has_main, has_sup = ctx.has
        return (g3[0] if has_main else None), g3[1], (g3[2] if has_sup else None), None, None


def loss_combine(s_main, s_un, s_sup, cnt, n, b, lambda_sup, lambda_cl):
    """(objective, detached [total, main, cl]) of the contrastive step from device scalars:
    s_main / n + lambda_cl * (s_un / b + lambda_sup * s_sup / max(cnt, 1)); s_main / s_sup may be
    None (no valid step / lambda_sup = 0), cnt is not differentiated."""
    consts = (1.0 / float(n) if n else 0.0, 1.0 / float(b), float(lambda_sup), float(lambda_cl))
    cnt = None if cnt is None else _c(cnt.detach().reshape(1))
    return _LossCombine.apply(s_main, s_un, s_sup, cnt, consts)


# ----------------------------------------------------------------------------------------
# The step's tail: clip_grad_norm_ + AdamW.step (v1_usertower_train.py:852-853), rsx_clip_adamw
_CLIP_ADAMW = os.environ.get("RSX_CLIP_ADAMW", "1") != "0"


def _adamw_native_ok(opt) -> bool:
    """torch.optim.AdamW configurations rsx_clip_adamw reproduces: no amsgrad / maximize /
    capturable / differentiable, float hyper-parameters, no step hooks."""
    if type(opt) is not torch.optim.AdamW or opt._optimizer_step_pre_hooks or opt._optimizer_step_post_hooks:
        return False
    from torch.optim import optimizer as _om
    if _om._global_optimizer_pre_hooks or _om._global_optimizer_post_hooks:
        return False
    if torch.get_default_dtype() != torch.float32:
        return False
    for g in opt.param_groups:
        if g.get("amsgrad") or g.get("maximize") or g.get("capturable") or g.get("differentiable"):
            return False
        if not g.get("decoupled_weight_decay", True):
            return False
        if any(isinstance(v, torch.Tensor) for v in (g["lr"], g["eps"], g["weight_decay"], *g["betas"])):
            return False
    return True


# per-optimizer pointer / size arrays of rsx_clip_adamw, reused while the parameter list, the
# clip set and the state tensors are the same objects (rebuilt otherwise; gradients every step)
_ADAMW_CACHE: "weakref.WeakKeyDictionary" = weakref.WeakKeyDictionary()


def module_params(model):
    """The set of model.parameters() (same members: every registered, non-None parameter of the
    module tree, each once) by a plain walk of _modules / _parameters: the clip set of the step,
    where only membership matters, without named_parameters()' prefix strings (~0.2 ms per step)."""
    out, seen, stack = [], set(), [model]
    while stack:
        m = stack.pop()
        for p in m._parameters.values():
            if p is not None and id(p) not in seen:
                seen.add(id(p))
                out.append(p)
        stack.extend(c for c in m._modules.values() if c is not None)
    return out


def clip_adamw_step(optimizer, clip_params, max_norm: float):
    """torch.nn.utils.clip_grad_norm_(clip_params, max_norm) followed by optimizer.step() for a
    torch.optim.AdamW, as two launches (rsx_clip_adamw) instead of torch's ~10 (per-tensor norms,
    stack, norm, clamp, foreach multiply, the AdamW kernels) and their ~1 ms of host time.
    Same state (optimizer.state[p]: step / exp_avg / exp_avg_sq, created as torch does), same
    in-place gradient scaling; the update follows torch's fused AdamW arithmetic. Returns the
    total norm (device scalar), or None when the optimizer or a tensor is one this does not
    handle (sparse / non-fp32 / non-contiguous / CPU, a clipped parameter the optimizer does not
    own): then nothing was changed and the caller runs torch's pair."""
    if not _CLIP_ADAMW or not _adamw_native_ok(optimizer):
        return None
    clip_ids = {id(p) for p in clip_params if p.grad is not None}
    items = []
    for g in optimizer.param_groups:
        for p in g["params"]:
            gr = p.grad
            if gr is None:
                continue
            if (gr.is_sparse or p.dtype != torch.float32 or gr.dtype != torch.float32 or p.device.type != "cuda"
                    or not p.is_contiguous() or not gr.is_contiguous() or gr.shape != p.shape):
                return None
            items.append((p, gr, g))
    if not items:
        return None
    if sum(1 for p, _, _ in items if id(p) in clip_ids) != len(clip_ids):
        return None
    N.ensure_device(items[0][0])
    state = optimizer.state
    for p, gr, g in items:
        st = state[p]
        if len(st) == 0:   # torch.optim.Adam._init_group
            st["step"] = (torch.zeros((), dtype=torch.float32, device=p.device) if g["fused"]
                          else torch.tensor(0.0, dtype=torch.float32))
            st["exp_avg"] = torch.zeros_like(p, memory_format=torch.preserve_format)
            st["exp_avg_sq"] = torch.zeros_like(p, memory_format=torch.preserve_format)
    sts = [state[p] for p, _, _ in items]
    sig = (tuple(id(p) for p, _, _ in items), frozenset(clip_ids),
           tuple((id(st["exp_avg"]), id(st["exp_avg_sq"]), id(st["step"])) for st in sts))
    c = _ADAMW_CACHE.get(optimizer)
    if c is None or c["sig"] != sig:
        m_l, v_l, dev_steps, cpu_steps = [], [], [], []
        for st in sts:
            m, v, s = st["exp_avg"], st["exp_avg_sq"], st["step"]
            if not (m.is_contiguous() and v.is_contiguous() and m.dtype == torch.float32 and v.dtype == torch.float32):
                return None
            m_l.append(m)
            v_l.append(v)
            (dev_steps if s.device.type == "cuda" else cpu_steps).append(s)
        n = len(items)
        numel = N.i64_array([p.numel() for p, _, _ in items])
        clip = (ctypes.c_int * n)(*[1 if id(p) in clip_ids else 0 for p, _, _ in items])
        steps_t = [st["step"] for st in sts]
        c = {"sig": sig, "n": n, "dev_steps": dev_steps, "cpu_steps": cpu_steps, "steps_t": steps_t,
             # the tensors are held so that the ids in sig cannot be reused by other objects
             "hold": (m_l, v_l, [p for p, _, _ in items]),
             "ps": N.ptr_array([p for p, _, _ in items]), "ms": N.ptr_array(m_l), "vs": N.ptr_array(v_l),
             "numel": numel, "clip": clip,
             "step_d": N.ptr_array([s if s.device.type == "cuda" else None for s in steps_t]) if dev_steps else None,
             "nbytes": N.lib().rsx_clip_adamw_workspace_bytes(n, numel, clip)}
        _ADAMW_CACHE[optimizer] = c
    n = c["n"]
    # the step counts first, as torch's AdamW does (one multi-tensor launch for device counts)
    if c["dev_steps"]:
        torch._foreach_add_(c["dev_steps"], 1.0)
    if c["cpu_steps"]:
        torch._foreach_add_(c["cpu_steps"], 1.0)
    gs = N.ptr_array([gr for _, gr, _ in items])
    step_h = (ctypes.c_float * n)(*[0.0 if s.device.type == "cuda" else float(s) for s in c["steps_t"]])
    lr = (ctypes.c_double * n)(*[g["lr"] for _, _, g in items])   # doubles, as torch's kernels take them
    wd = (ctypes.c_double * n)(*[g["weight_decay"] for _, _, g in items])
    b1 = (ctypes.c_double * n)(*[g["betas"][0] for _, _, g in items])
    b2 = (ctypes.c_double * n)(*[g["betas"][1] for _, _, g in items])
    eps = (ctypes.c_double * n)(*[g["eps"] for _, _, g in items])
    dev = items[0][0].device
    nbytes = c["nbytes"]
    ws = torch.empty(nbytes, device=dev, dtype=torch.uint8)
    norm = torch.empty((), device=dev, dtype=torch.float32)
    rc = N.lib().rsx_clip_adamw(n, c["ps"], gs, c["ms"], c["vs"], c["numel"], c["clip"], step_h, c["step_d"], lr, wd,
                                b1, b2, eps, float(max_norm), N.ptr(ws), nbytes, N.ptr(norm), N.stream())
    N.check(rc, "clip_adamw")
    optimizer._opt_called = True   # what torch's step wrapper records (LR schedulers check it)
    return norm


def zero_grad_(optimizer) -> None:
    """optimizer.zero_grad(set_to_none=True) without the profiler record_function around it."""
    for g in optimizer.param_groups:
        for p in g["params"]:
            p.grad = None


# ----------------------------------------------------------------------------------------
# Static-profile embeddings (several tiny gated tables, concatenated): rsx_static_embed_*
class _StaticEmbed(torch.autograd.Function):
    @staticmethod
    def forward(ctx, gate, ids, padding_idx, *tables):
        N.ensure_device(gate)
        ids = [_c(t) for t in ids]
        tables = [_c(t) for t in tables]
        B = ids[0].shape[0]
        dims = [t.shape[1] for t in tables]
        out = torch.empty(B, sum(dims), device=gate.device, dtype=torch.float32)
        gate = _c(gate)
        rc = N.lib().rsx_static_embed_fwd(N.ptr_array(ids), N.ptr_array(tables),
                                          N.i64_array([t.shape[0] for t in tables]), N.i64_array(dims), len(tables),
                                          N.ptr(gate), B, N.ptr(out), out.stride(0), N.stream())
        N.check(rc, "static_embed_fwd")
        ctx.save_for_backward(gate, *ids, *tables)
        ctx.cfg = (len(tables), list(padding_idx))
        return out

    @staticmethod
    def backward(ctx, dout):
        nt, pad = ctx.cfg
        saved = ctx.saved_tensors
        gate, ids, tables = saved[0], list(saved[1:1 + nt]), list(saved[1 + nt:1 + 2 * nt])
        need = ctx.needs_input_grad
        dgate, *dtabs = _empty_group([gate if need[0] else None] +
                                     [t if need[3 + j] else None for j, t in enumerate(tables)])
        dout = _c(dout)
        B = ids[0].shape[0]
        rows = N.i64_array([t.shape[0] for t in tables])
        dims = N.i64_array([t.shape[1] for t in tables])
        nws = N.lib().rsx_static_embed_bwd_workspace_floats(B, nt, rows, dims)
        ws = torch.empty(nws, device=dout.device, dtype=torch.float32)
        rc = N.lib().rsx_static_embed_bwd(N.ptr_array(ids), N.ptr_array(tables), rows, dims, N.i64_array(pad), nt,
                                          N.ptr(gate), N.ptr(dout), dout.stride(0), B, B, N.ptr_array(dtabs),
                                          N.ptr(dgate), 0, N.ptr(ws), nws, N.stream())  # written
        N.check(rc, "static_embed_bwd")
        return (dgate, None, None, *dtabs)


def static_embed(ids, tables, gate, padding_idx=None):
    """cat_j(tables[j][ids[j]] * gate[j]) -> [B, sum_j dim_j] (nn.Embedding padding_idx
    semantics for the gradient)."""
    if padding_idx is None:
        padding_idx = [-1] * len(tables)
    padding_idx = [(-1 if p is None else int(p)) for p in padding_idx]
    return _StaticEmbed.apply(gate, list(ids), padding_idx, *tables)


# ----------------------------------------------------------------------------------------
# A4: the static profile as one native call per direction (rsx_static_profile_*)
_SP_IDS, _SP_TABLES, _SP_GATE, _SP_N = 0, 16, 32, 40


class _StaticProfile(torch.autograd.Function):
    @staticmethod
    def forward(ctx, cfg, static_gate, cont, wc, bc, wm, bm, ln_w, ln_b, *tables):
        ids, pads, eps, p_drop, seed, U = cfg
        N.ensure_device(static_gate)
        ids = [_c(t) for t in ids]
        tables = [_c(t) for t in tables]
        params = [_c(t) for t in (static_gate, cont, wc, bc, wm, bm, ln_w, ln_b)]
        src = ids[0].shape[0]
        nt = len(tables)
        ptrs = [None] * _SP_N
        ptrs[_SP_IDS:_SP_IDS + nt] = ids
        ptrs[_SP_TABLES:_SP_TABLES + nt] = tables
        ptrs[_SP_GATE:_SP_N] = params
        p_arr = N.ptr_array(ptrs)
        dims = N.i64_array([U, nt, cont.shape[1], wc.shape[0], wm.shape[1], src] + [t.shape[0] for t in tables]
                           + [t.shape[1] for t in tables] + list(pads))
        lib = N.lib()
        arena = torch.empty(lib.rsx_static_profile_arena_bytes(U), device=static_gate.device, dtype=torch.uint8)
        out = torch.empty(U, wm.shape[0], device=static_gate.device, dtype=torch.float32)
        rc = lib.rsx_static_profile_fwd(p_arr, dims, eps, p_drop, seed, N.ptr(arena), arena.numel(), N.ptr(out),
                                        N.stream())
        N.check(rc, "static_profile_fwd")
        # the kernel range-checks the nine ids (an out-of-range id reads and scatters row 0 and sets
        # the flag in the arena's first int32): raised as IndexError at the next poll / check
        _STATIC_IDS.watch(arena[:4].view(torch.int32))
        # the parameters and tables through autograd's saved tensors, so an in-place change between
        # forward and backward raises instead of the backward reading the new values
        ctx.save_for_backward(*params, *tables)
        ctx.keep = (p_arr, dims, ptrs, arena, p_drop, seed, U)
        return out

    @staticmethod
    def backward(ctx, dout):
        ctx.saved_tensors  # noqa: B018 -- the version check of the saved parameters and tables
        p_arr, dims, ptrs, arena, p_drop, seed, U = ctx.keep
        nt = len(ctx.needs_input_grad) - 9
        likes = [ptrs[_SP_GATE]] + [None] + ptrs[_SP_GATE + 2:_SP_N] + ptrs[_SP_TABLES:_SP_TABLES + nt]
        if U == 0:
            grads = [None if t is None else torch.zeros_like(t) for t in likes]
        else:
            grads = _empty_group(likes)
            g_ptrs = [None] * _SP_N
            g_ptrs[_SP_GATE:_SP_N] = grads[:8]
            g_ptrs[_SP_TABLES:_SP_TABLES + nt] = grads[8:]
            lib = N.lib()
            nws = lib.rsx_static_profile_bwd_workspace_bytes(U)
            ws = torch.empty(nws, device=dout.device, dtype=torch.uint8)
            rc = lib.rsx_static_profile_bwd(p_arr, dims, p_drop, seed, N.ptr(arena), N.ptr(_c(dout)),
                                            N.ptr_array(g_ptrs), N.ptr(ws), nws, N.stream())
            N.check(rc, "static_profile_bwd")
        return (None, *grads)


def static_profile(model, ids, cont_feats, p_drop, rows=None):
    """SASRecUserTower phase 2 (v1_refine_usertower.py:472-494): sigmoid(static_gate), the nine
    gated lookups, relu(cont_proj(cont)) * u_g[9], static_mlp (Linear + LayerNorm + GELU +
    Dropout) -> [rows, 128], as rsx_static_profile_fwd / _bwd (dropout: counter-hash mask).
    ids (nine int64 [B]) / cont_feats [B, 4] hold B users; rows (default B, a multiple of B):
    output row r is user r % B (the two dropout views of the contrastive step: rows = 2B)."""
    B = ids[0].shape[0]
    rows = B if rows is None else int(rows)
    if B == 0 or rows % B:
        raise ValueError(f"static_profile: rows ({rows}) must be a positive multiple of the users ({B})")
    embs = [model.age_emb, model.price_emb, model.cnt_emb, model.recency_emb, model.channel_emb,
            model.club_status_emb, model.news_freq_emb, model.fn_emb, model.active_emb]
    lin, ln = model.static_mlp[0], model.static_mlp[1]
    seed = next_seed() if p_drop > 0 else 0
    pads = [(-1 if e.padding_idx is None else int(e.padding_idx)) for e in embs]
    cfg = ([t.to(torch.int64) for t in ids], pads, float(ln.eps), float(p_drop), seed, rows)
    return _StaticProfile.apply(cfg, model.static_gate, cont_feats.to(torch.float32), model.cont_proj.weight,
                                model.cont_proj.bias,
                                lin.weight, lin.bias, ln.weight, ln.bias, *[e.weight for e in embs])


# ----------------------------------------------------------------------------------------
# LayerNorm (+ residual add + dropout before it, + GELU after it): rsx_ln_fwd / rsx_ln_bwd
ACT_GELU_ERF = 2


def _ln_bwd(s, mean, rstd, w, b, act, dy, ds_in, p_drop, seed, want_dx, want_dres, want_w, want_b):
    T, D = s.shape
    dx = torch.empty_like(s) if want_dx or want_dres else None
    dres = torch.empty_like(s) if want_dres else None
    dw = torch.empty(D, device=s.device, dtype=torch.float32) if want_w else None
    db = torch.empty(D, device=s.device, dtype=torch.float32) if want_b else None
    nws = N.lib().rsx_ln_bwd_workspace_floats(T, D)
    ws = torch.empty(nws, device=s.device, dtype=torch.float32) if (want_w or want_b) else None
    with timed("ln_bwd"):
        rc = N.lib().rsx_ln_bwd(N.ptr(s), N.ptr(mean), N.ptr(rstd), N.ptr(w), N.ptr(b), act, N.ptr(_c(dy)),
                                N.ptr(None if ds_in is None else _c(ds_in)), p_drop, seed, T, D, N.ptr(dx),
                                N.ptr(dres), N.ptr(dw), N.ptr(db), N.ptr(ws), nws if ws is not None else 0,
                                N.stream())
    N.check(rc, "ln_bwd")
    return dx, dres, dw, db


class _LayerNorm(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, w, b, eps, act):
        N.ensure_device(x)
        x = _c(x)
        T, D = x.shape
        y = torch.empty_like(x)
        mean = torch.empty(T, device=x.device, dtype=torch.float32)
        rstd = torch.empty_like(mean)
        with timed("ln_fwd"):
            rc = N.lib().rsx_ln_fwd(N.ptr(x), None, 0.0, 0, N.ptr(w), N.ptr(b), eps, act, T, D, None, N.ptr(y),
                                    N.ptr(mean), N.ptr(rstd), N.stream())
        N.check(rc, "ln_fwd")
        ctx.save_for_backward(x, mean, rstd, w, b)
        ctx.act = act
        return y

    @staticmethod
    def backward(ctx, dy):
        x, mean, rstd, w, b = ctx.saved_tensors
        need = ctx.needs_input_grad
        dx, _, dw, db = _ln_bwd(x, mean, rstd, w, b, ctx.act, dy, None, 0.0, 0, need[0], False, need[1], need[2])
        return dx, dw, db, None, None


class _AddLayerNorm(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, res, w, b, eps, p_drop, seed):
        N.ensure_device(x)
        x = _c(x)
        res = _c(res)
        T, D = x.shape
        s = torch.empty_like(x)
        y = torch.empty_like(x)
        mean = torch.empty(T, device=x.device, dtype=torch.float32)
        rstd = torch.empty_like(mean)
        with timed("ln_fwd"):
            rc = N.lib().rsx_ln_fwd(N.ptr(x), N.ptr(res), p_drop, seed, N.ptr(w), N.ptr(b), eps, 0, T, D, N.ptr(s),
                                    N.ptr(y), N.ptr(mean), N.ptr(rstd), N.stream())
        N.check(rc, "ln_fwd")
        ctx.save_for_backward(s, mean, rstd, w, b)
        ctx.cfg = (p_drop, seed)
        return s, y

    @staticmethod
    def backward(ctx, ds, dy):
        s, mean, rstd, w, b = ctx.saved_tensors
        p_drop, seed = ctx.cfg
        need = ctx.needs_input_grad
        if dy is None:
            dy = torch.zeros_like(s)
        dx, dres, dw, db = _ln_bwd(s, mean, rstd, w, b, 0, dy, ds, p_drop, seed, need[0], need[1], need[2], need[3])
        return dx, dres, dw, db, None, None, None


class _LayerNormPass(torch.autograd.Function):
    """(x, LayerNorm(x)): the first norm1 of a norm_first encoder, whose input also feeds the
    residual. The backward adds the residual-path gradient inside the LayerNorm backward
    (ds_in) instead of autograd's separate add of two [T, D] gradients."""

    @staticmethod
    def forward(ctx, x, w, b, eps):
        N.ensure_device(x)
        T, D = x.shape
        y = torch.empty_like(x)
        mean = torch.empty(T, device=x.device, dtype=torch.float32)
        rstd = torch.empty_like(mean)
        with timed("ln_fwd"):
            rc = N.lib().rsx_ln_fwd(N.ptr(x), None, 0.0, 0, N.ptr(w), N.ptr(b), eps, 0, T, D, None, N.ptr(y),
                                    N.ptr(mean), N.ptr(rstd), N.stream())
        N.check(rc, "ln_fwd")
        ctx.save_for_backward(x, mean, rstd, w, b)
        return x.view_as(x), y

    @staticmethod
    def backward(ctx, dx_pass, dy):
        x, mean, rstd, w, b = ctx.saved_tensors
        need = ctx.needs_input_grad
        if dy is None:
            return dx_pass, None, None, None
        dx, _, dw, db = _ln_bwd(x, mean, rstd, w, b, 0, dy, dx_pass, 0.0, 0, need[0], False, need[1], need[2])
        return dx, dw, db, None


def layer_norm_pass(x, weight, bias, eps=1e-5):
    """(x, LayerNorm(x)) with the residual gradient of x folded into the LayerNorm backward."""
    shp = x.shape
    x2, y = _LayerNormPass.apply(_c(x.reshape(-1, shp[-1])), weight, bias, float(eps))
    return x2.reshape(shp), y.reshape(shp)


class _AddDropout(torch.autograd.Function):
    """s = x + dropout_p(res) in one pass (rsx_ln_fwd's add-only form); backward dx = ds,
    dres = mask(ds) (rsx_dropout_bwd, the same counter hash)."""

    @staticmethod
    def forward(ctx, x, res, p_drop, seed):
        N.ensure_device(x)
        T, D = x.shape
        s = torch.empty_like(x)
        rc = N.lib().rsx_ln_fwd(N.ptr(x), N.ptr(res), p_drop, seed, None, None, 0.0, 0, T, D, N.ptr(s), None,
                                None, None, N.stream())
        N.check(rc, "ln_fwd(add)")
        ctx.cfg = (p_drop, seed, T, D)
        return s

    @staticmethod
    def backward(ctx, ds):
        p_drop, seed, T, D = ctx.cfg
        ds = _c(ds)
        dres = None
        if ctx.needs_input_grad[1]:
            dres = torch.empty_like(ds)
            rc = N.lib().rsx_dropout_bwd(N.ptr(ds), T, D, p_drop, seed, N.ptr(dres), N.stream())
            N.check(rc, "dropout_bwd")
        return ds, dres, None, None


def add_dropout(x, res, p_drop=0.0, training=True):
    """x + F.dropout(res, p_drop, training) as one kernel (counter-hash mask; p = 0 in eval)."""
    p = float(p_drop) if training else 0.0
    shp = x.shape
    seed = next_seed() if p > 0 else 0
    s = _AddDropout.apply(_c(x.reshape(-1, shp[-1])), _c(res.reshape(-1, shp[-1])), p, seed)
    return s.reshape(shp)


def layer_norm(x, weight, bias, eps=1e-5, act=0):
    """act(LayerNorm(x)) over the last dim (act 0 none / ACT_GELU_ERF)."""
    shp = x.shape
    y = _LayerNorm.apply(x.reshape(-1, shp[-1]), weight, bias, float(eps), int(act))
    return y.reshape(shp)


@torch.no_grad()
def add_layer_norm_infer(x, res, weight, bias, eps=1e-5):
    """LayerNorm(x + res) forward only (no statistics saved, the sum not written): inference,
    e.g. BERT's post-norm residuals in item_tower.bert_cls_packed. Hidden up to 1024."""
    N.ensure_device(x)
    x = _c(x)
    res = _c(res)
    T, D = x.shape
    y = torch.empty_like(x)
    rc = N.lib().rsx_ln_fwd(N.ptr(x), N.ptr(res), 0.0, 0, N.ptr(weight), N.ptr(bias), float(eps), 0, T, D, None,
                            N.ptr(y), None, None, N.stream())
    N.check(rc, "ln_fwd(add, inference)")
    return y


def add_layer_norm(x, res, weight, bias, eps=1e-5, p_drop=0.0):
    """(s, LayerNorm(s)) with s = x + dropout(res): the residual add of a norm_first encoder
    layer fused with the next LayerNorm."""
    shp = x.shape
    seed = next_seed() if p_drop > 0 else 0
    s, y = _AddLayerNorm.apply(x.reshape(-1, shp[-1]), res.reshape(-1, shp[-1]), weight, bias, float(eps),
                               float(p_drop), seed)
    return s.reshape(shp), y.reshape(shp)


# ----------------------------------------------------------------------------------------
# Token-level linear layers: forward / dX on rsx_gemm_x3, dW / db on rsx_linear_wgrad(_x3)
# Token-linear GEMM precision: "bf16x3" = rsx_gemm_x3 / rsx_linear_wgrad_x3 (hi/lo bf16 split
# on the bf16 MFMA, ~2^-17 relative error per product), "fp32" = the library fp32 GEMM for the
# forward / input gradient and the fp32-MFMA rsx_linear_wgrad. RSX_GEMM_PRECISION selects.
GEMM_PRECISIONS = ("fp32", "bf16x3")
_gemm_precision = os.environ.get("RSX_GEMM_PRECISION", "bf16x3")
EPI_BIAS, EPI_GELU_DROP, EPI_DGELU_DROP = 0, 1, 2


def set_gemm_precision(p: str) -> str:
    """Set the token-linear GEMM precision ("fp32" | "bf16x3"); returns the previous mode."""
    global _gemm_precision
    if p not in GEMM_PRECISIONS:
        raise ValueError(f"precision must be one of {sorted(GEMM_PRECISIONS)}")
    prev, _gemm_precision = _gemm_precision, p
    return prev


def _x3_ok(m_out: int, k_in: int) -> bool:
    return _gemm_precision == "bf16x3" and m_out % 128 == 0 and k_in % 32 == 0


def gemm_x3(a, b, bias=None, epi=EPI_BIAS, aux=None, p_drop=0.0, seed=0, tag=None):
    """epi(a [M, K] @ b [N, K]^T + bias) on rsx_gemm_x3 (N % 128 == 0, K % 32 == 0).
    EPI_GELU_DROP returns dropout(gelu(pre)) and writes gelu'(pre) into aux;
    EPI_DGELU_DROP returns (a @ b^T) * keep / (1 - p) * aux."""
    a = _c(a)
    b = _c(b)
    M, K = a.shape
    n = b.shape[0]
    out = torch.empty(M, n, device=a.device, dtype=torch.float32)
    if M == 0:
        return out
    nws = N.lib().rsx_gemm_x3_split_floats(M, n, K)  # > 0: split-K for a shape with fewer tiles than CUs
    ws = torch.empty(nws, device=a.device, dtype=torch.float32) if nws > 0 else None
    with timed(tag or "gemm_x3"):
        rc = N.lib().rsx_gemm_x3_ws(N.ptr(a), a.stride(0), N.ptr(b), b.stride(0),
                                    N.ptr(None if bias is None else _c(bias)), M, n, K, epi, N.ptr(aux),
                                    0 if aux is None else aux.stride(0), float(p_drop), int(seed), N.ptr(out),
                                    out.stride(0), N.ptr(ws), nws, N.stream())
    N.check(rc, "gemm_x3")
    return out


def _tn_ok(w) -> bool:
    """rsx_gemm_x3_tn takes W [out, in] as stored for dX = dY W (weight-stationary path)."""
    return (_gemm_precision == "bf16x3" and w.shape[0] in (128, 256, 384) and w.shape[1] % 128 == 0
            and w.stride(1) == 1 and w.stride(0) % 4 == 0)


def gemm_x3_tn(a, w, epi=EPI_BIAS, aux=None, p_drop=0.0, seed=0, tag=None):
    """epi(a [M, K] @ w [K, N]) on rsx_gemm_x3_tn: the input gradient dY W of a token linear with W
    as stored ([out, in], K = out in {128, 256, 384}, N = in % 128 == 0), no transposed copy;
    EPI_DGELU_DROP as gemm_x3."""
    a = _c(a)
    M, K = a.shape
    n = w.shape[1]
    out = torch.empty(M, n, device=a.device, dtype=torch.float32)
    if M == 0:
        return out
    with timed(tag or "gemm_x3"):
        rc = N.lib().rsx_gemm_x3_tn(N.ptr(a), a.stride(0), N.ptr(w), w.stride(0), None, M, n, K, epi, N.ptr(aux),
                                    0 if aux is None else aux.stride(0), float(p_drop), int(seed), N.ptr(out),
                                    out.stride(0), N.stream())
    N.check(rc, "gemm_x3_tn")
    return out


def _dx(dy, w, tag="tok_linear_dx"):
    """dX = dY W of a token linear (rsx_gemm_x3_tn when the shape allows, else a transposed copy)."""
    if _tn_ok(w):
        return gemm_x3_tn(dy, w, tag=tag)
    return gemm_x3(dy, w.t(), tag=tag)


def linear_wgrad(dy, x, weight_shape, need_bias, tag="linear_wgrad"):
    """(dW, db) of y = x W^T + b over the token axis: split-K over tokens, deterministic."""
    N.ensure_device(dy)
    dy = _c(dy)
    x = _c(x)
    t, n = dy.shape
    k = x.shape[1]
    assert (n, k) == tuple(weight_shape)
    nws = N.lib().rsx_linear_wgrad_workspace_floats(t, n, k)
    ws = torch.empty(nws, device=dy.device, dtype=torch.float32)
    dw = torch.empty(n, k, device=dy.device, dtype=torch.float32)
    db = torch.empty(n, device=dy.device, dtype=torch.float32) if need_bias else None
    fn = N.lib().rsx_linear_wgrad_x3 if _gemm_precision == "bf16x3" else N.lib().rsx_linear_wgrad
    with timed(tag):
        rc = fn(N.ptr(dy), dy.stride(0), N.ptr(x), x.stride(0), t, n, k, N.ptr(dw), dw.stride(0), N.ptr(db), 0,
                N.ptr(ws), nws, N.stream())
    N.check(rc, "linear_wgrad")
    return dw, db


class _TokLinear(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, weight, bias):
        ctx.save_for_backward(x, weight)
        ctx.has_bias = bias is not None
        if _x3_ok(weight.shape[0], weight.shape[1]):
            return gemm_x3(x, weight, bias, tag="tok_linear_fwd")
        return torch.nn.functional.linear(x, weight, bias)

    @staticmethod
    def backward(ctx, dy):
        x, weight = ctx.saved_tensors
        dy = _c(dy)
        dx = None
        if ctx.needs_input_grad[0]:
            if _x3_ok(weight.shape[1], weight.shape[0]):
                dx = _dx(dy, weight)
            else:
                dx = dy @ weight
        dw = db = None
        if ctx.needs_input_grad[1] or (ctx.has_bias and ctx.needs_input_grad[2]):
            dw, db = linear_wgrad(dy, x, weight.shape, ctx.has_bias and ctx.needs_input_grad[2])
        return dx, dw, db


class _LinearAddLayerNorm(torch.autograd.Function):
    """(s, LayerNorm(s)), s = x + dropout(a W^T + b): rsx_gemm_x3_addln (the add and the
    LayerNorm in the GEMM's epilogue; the projection itself is never written). Backward: the
    add + LayerNorm backward (rsx_ln_bwd, whose dres is the projection's gradient), then dA on
    rsx_gemm_x3 and dW / db on the split-K weight-gradient kernel, as _TokLinear."""

    @staticmethod
    def forward(ctx, x, a, weight, bias, w, b, eps, p_drop, seed):
        T, D = x.shape
        s = torch.empty_like(x)
        y = torch.empty_like(x)
        mean = torch.empty(T, device=x.device, dtype=torch.float32)
        rstd = torch.empty_like(mean)
        with timed("tok_linear_addln"):
            rc = N.lib().rsx_gemm_x3_addln(N.ptr(a), a.stride(0), N.ptr(weight), weight.stride(0), N.ptr(bias), T, D,
                                           a.shape[1], N.ptr(x), x.stride(0), p_drop, seed, N.ptr(w), N.ptr(b), eps,
                                           N.ptr(s), s.stride(0), N.ptr(y), y.stride(0), N.ptr(mean), N.ptr(rstd),
                                           N.stream())
        N.check(rc, "gemm_x3_addln")
        ctx.save_for_backward(a, weight, s, mean, rstd, w, b)
        ctx.cfg = (p_drop, seed, bias is not None)
        return s, y

    @staticmethod
    def backward(ctx, ds, dy):
        a, weight, s, mean, rstd, w, b = ctx.saved_tensors
        p_drop, seed, has_bias = ctx.cfg
        need = ctx.needs_input_grad
        if dy is None:
            dy = torch.zeros_like(s)
        dx, dres, dw, db = _ln_bwd(s, mean, rstd, w, b, 0, dy, ds, p_drop, seed, need[0], True, need[4], need[5])
        da = _dx(dres, weight) if need[1] else None
        dwt = dbt = None
        if need[2] or (has_bias and need[3]):
            dwt, dbt = linear_wgrad(dres, a, weight.shape, has_bias and need[3])
        return dx, da, dwt, dbt, dw, db, None, None, None


def linear_add_layer_norm(x, a, weight, bias, ln_weight, ln_bias, eps=1e-5, p_drop=0.0):
    """(s, LayerNorm(s)) with s = x + dropout(linear(a, weight, bias)): a norm_first encoder
    layer's attention out-projection, residual add and the LayerNorm after it in one kernel
    (bf16x3 mode, D = 128, K 128 or 256); otherwise linear_tok + add_layer_norm."""
    shp = x.shape
    D = shp[-1]
    if not (_x3_ok(weight.shape[0], weight.shape[1]) and D == 128 and weight.shape[0] == 128
            and weight.shape[1] in (128, 256) and x.numel() > 0):
        return add_layer_norm(x, linear_tok(a, weight, bias), ln_weight, ln_bias, eps, p_drop)
    N.ensure_device(x)
    seed = next_seed() if p_drop > 0 else 0
    s, y = _LinearAddLayerNorm.apply(_c(x.reshape(-1, D)), _c(a.reshape(-1, a.shape[-1])), _c(weight), bias,
                                     ln_weight, ln_bias, float(eps), float(p_drop), seed)
    return s.reshape(shp), y.reshape(shp)


def linear_tok(x, weight, bias=None):
    """F.linear over a token axis (x [..., K]) whose weight/bias gradients come from the
    split-K rsx_linear_wgrad kernel instead of the library GEMM (T >> N, K); forward and
    input gradient on rsx_gemm_x3 when the shapes allow (bf16x3 mode). GPU tensors only."""
    N.ensure_device(x)
    shp = x.shape
    x2 = _c(x.reshape(-1, shp[-1]))
    if x2.shape[0] == 0 or shp[-1] % 16 or weight.shape[0] % 16:
        return torch.nn.functional.linear(x, weight, bias)
    y = _TokLinear.apply(x2, weight, bias)
    return y.reshape(*shp[:-1], weight.shape[0])


class _ProfileLinear(torch.autograd.Function):
    """h[t] = x[t] W[:, :D]^T + (profile W[:, D:]^T + b)[user(t)]: nn.Linear(2D -> N) applied
    to cat(x_tok, profile[user]) without materialising the concatenation or the broadcast
    (v1_refine_usertower.py:498-505, output_proj[0] on the packed tokens). Forward: the small
    per-user GEMM, then the token GEMM with the per-user rows added in its epilogue
    (rsx_gemm_x3_rowadd). Backward: dX on rsx_gemm_x3; the per-user gradient is a segmented
    sum over each user's contiguous tokens (rsx_segment_sum_rows, no atomics); both weight
    halves and the bias from the split-K weight-gradient kernel, written into one [N, 2D]
    gradient (no slice / concatenation kernels)."""

    @staticmethod
    def forward(ctx, x, profile, weight, bias, tok_user, seg):
        D = x.shape[1]
        n = weight.shape[0]
        wp = weight[:, D:]
        prof = gemm_x3(profile, wp, bias, tag="tok_linear_fwd") if _x3_ok(n, D) else \
            torch.addmm(bias, profile, wp.t())
        h = torch.empty(x.shape[0], n, device=x.device, dtype=torch.float32)
        with timed("tok_linear_fwd"):
            rc = N.lib().rsx_gemm_x3_rowadd(N.ptr(x), x.stride(0), N.ptr(weight), weight.stride(0), None,
                                            x.shape[0], n, D, N.ptr(prof), prof.stride(0), N.ptr(tok_user),
                                            N.ptr(h), h.stride(0), N.stream())
        N.check(rc, "gemm_x3_rowadd")
        ctx.save_for_backward(x, profile, weight, seg)
        return h

    @staticmethod
    def backward(ctx, dh):
        x, profile, weight, seg = ctx.saved_tensors
        dh = _c(dh)
        D = x.shape[1]
        n = weight.shape[0]
        U = profile.shape[0]
        dprof = torch.empty(U, n, device=dh.device, dtype=torch.float32)
        rc = N.lib().rsx_segment_sum_rows(N.ptr(dh), dh.stride(0), None, N.ptr(seg), None, U, n, None, -1,
                                          N.ptr(dprof), dprof.stride(0), 0, N.stream())
        N.check(rc, "segment_sum_rows(profile)")
        dx = dprofile = None
        if ctx.needs_input_grad[0]:
            dx = _dx(dh, weight[:, :D])
        if ctx.needs_input_grad[1]:
            dprofile = _dx(dprof, weight[:, D:]) if _x3_ok(D, n) else \
                dprof @ weight[:, D:]
        dw = torch.empty_like(weight)
        db = torch.empty(n, device=dh.device, dtype=torch.float32)
        _wgrad_into(dh, x, dw[:, :D], None)
        _wgrad_into(dprof, profile, dw[:, D:], db)
        return dx, dprofile, dw, db, None, None


def _wgrad_into(dy, x, dw_view, db):
    """dW (+ db) of y = x W^T + b written into a (row-strided) view: rsx_linear_wgrad(_x3)."""
    t, n = dy.shape
    k = x.shape[1]
    nws = N.lib().rsx_linear_wgrad_workspace_floats(t, n, k)
    ws = torch.empty(nws, device=dy.device, dtype=torch.float32)
    fn = N.lib().rsx_linear_wgrad_x3 if _gemm_precision == "bf16x3" else N.lib().rsx_linear_wgrad
    with timed("linear_wgrad"):
        rc = fn(N.ptr(dy), dy.stride(0), N.ptr(_c(x)), x.stride(0), t, n, k, N.ptr(dw_view), dw_view.stride(0),
                N.ptr(db), 0, N.ptr(ws), nws, N.stream())
    N.check(rc, "linear_wgrad")


def profile_linear(x, profile, weight, bias, tok_user, seg):
    """x [T, D] packed tokens, profile [U, D] per user, weight [N, 2D], bias [N], tok_user [T]
    int64 (user of each token, non-decreasing), seg [U + 1] int64 token offsets of the users.
    Returns [T, N] = F.linear(cat(x, profile[tok_user]), weight, bias)."""
    N.ensure_device(x)
    D = x.shape[1]
    n = weight.shape[0]
    if (x.shape[0] == 0 or weight.shape[1] != 2 * D or D not in (128, 256) or n % 128 or weight.stride(1) != 1
            or weight.stride(0) % 4 or _gemm_precision != "bf16x3"):
        return linear_tok(x, weight[:, :D]) + torch.nn.functional.linear(profile, weight[:, D:], bias)[tok_user]
    return _ProfileLinear.apply(_c(x), _c(profile), weight, bias, _c(tok_user), _c(seg))


class _FFN(torch.autograd.Function):
    """linear2(dropout(gelu(linear1(h)))) with the GELU and the dropout in the GEMM epilogues
    (rsx_gemm_x3 EPI_GELU_DROP forward, EPI_DGELU_DROP for the backward through them)."""

    @staticmethod
    def forward(ctx, h, w1, b1, w2, b2, p_drop, seed):
        h = _c(h)
        ggrad = torch.empty(h.shape[0], w1.shape[0], device=h.device, dtype=torch.float32)  # gelu'(pre)
        act = gemm_x3(h, w1, b1, EPI_GELU_DROP, ggrad, p_drop, seed, tag="ffn_fwd1")
        f = gemm_x3(act, w2, b2, tag="ffn_fwd2")
        ctx.save_for_backward(h, w1, w2, ggrad, act)
        ctx.cfg = (p_drop, seed, b1 is not None, b2 is not None)
        return f

    @staticmethod
    def backward(ctx, df):
        h, w1, w2, ggrad, act = ctx.saved_tensors
        p_drop, seed, has_b1, has_b2 = ctx.cfg
        df = _c(df)
        need = ctx.needs_input_grad
        if _tn_ok(w2):
            dpre = gemm_x3_tn(df, w2, EPI_DGELU_DROP, ggrad, p_drop, seed, tag="ffn_dpre")
        else:
            dpre = gemm_x3(df, w2.t(), None, EPI_DGELU_DROP, ggrad, p_drop, seed, tag="ffn_dpre")
        dw2 = db2 = dw1 = db1 = None
        if need[3] or need[4]:
            dw2, db2 = linear_wgrad(df, act, w2.shape, has_b2 and need[4])
        if need[1] or need[2]:
            dw1, db1 = linear_wgrad(dpre, h, w1.shape, has_b1 and need[2])
        dh = _dx(dpre, w1, tag="ffn_dh") if need[0] else None
        return dh, dw1, db1, dw2, db2, None, None


def ffn(h, w1, b1, w2, b2, p_drop=0.0, training=True):
    """linear2(dropout(gelu(linear1(h)))) over a token axis (nn.TransformerEncoderLayer's
    feed-forward block, activation="gelu"). bf16x3 mode with GEMM-shaped widths: two fused
    GEMM launches forward, three plus two weight gradients backward; otherwise the unfused ops."""
    p = float(p_drop) if training else 0.0
    shp = h.shape
    h2 = h.reshape(-1, shp[-1])
    if (h2.is_cuda and h2.shape[0] > 0 and _x3_ok(w1.shape[0], w1.shape[1]) and _x3_ok(w2.shape[0], w2.shape[1])
            and _x3_ok(w2.shape[1], w2.shape[0]) and _x3_ok(w1.shape[1], w1.shape[0])):
        seed = next_seed() if p > 0 else 0
        f = _FFN.apply(h2, w1, b1, w2, b2, p, seed)
        return f.reshape(*shp[:-1], w2.shape[0])
    return linear_tok(torch.nn.functional.dropout(torch.nn.functional.gelu(linear_tok(h, w1, b1)), p, training),
                      w2, b2)


# ----------------------------------------------------------------------------------------
# A2 + A3 + A4: the user tower's packed-token training program as one native call per direction
# (rsx_tower_fwd / rsx_tower_bwd, csrc/tower.hip). RSX_TOWER_NATIVE=0 keeps the per-op path.
_TOWER_NATIVE = os.environ.get("RSX_TOWER_NATIVE", "1") != "0"


def tower_params(model):
    """SASRecUserTower parameters in rsx_tower_* order (include/recsys_amd.h RSX_TW_ITEM_PROJ ..)."""
    ps = [model.item_proj.weight, model.item_proj.bias, model.item_id_emb.weight, model.time_emb.weight,
          model.type_emb.weight, model.color_emb.weight, model.graphic_emb.weight, model.section_emb.weight,
          model.pos_emb.weight, model.emb_ln.weight, model.emb_ln.bias]
    for layer in model.transformer_encoder.layers:
        sa = layer.self_attn
        ps += [layer.norm1.weight, layer.norm1.bias, sa.in_proj_weight, sa.in_proj_bias, sa.out_proj.weight,
               sa.out_proj.bias, layer.norm2.weight, layer.norm2.bias, layer.linear1.weight, layer.linear1.bias,
               layer.linear2.weight, layer.linear2.bias]
    op = model.output_proj
    ps += [op[0].weight, op[0].bias, op[1].weight, op[1].bias, op[3].weight, op[3].bias]
    return ps


def tower_native_ok(model, packed, pv):
    """Whether rsx_tower_* runs exactly what forward_packed's per-op path runs: bf16x3 token linears
    and attention, d_model 128 with 4 heads and a 256-wide feed-forward, every parameter trained,
    fp32 contiguous rows, the item-id gradient plan present. Returns the parameter list in
    rsx_tower_* order (truthy; tower_packed takes it) or None."""
    if not (_TOWER_NATIVE and _gemm_precision == "bf16x3" and _mha_precision == "bf16x3" and _ADDLN_ON):
        return None
    if getattr(packed, "item_seg", None) is None or not pv.is_cuda:
        return None
    layers = model.transformer_encoder.layers
    if model.d_model != 128 or not (1 <= len(layers) <= 8) or model.pos_emb.weight.shape[0] > 64:
        return None
    for layer in layers:
        if (layer.self_attn.num_heads != 4 or layer.linear1.out_features != 256 or not layer.norm_first
                or layer.activation_relu_or_gelu != 2):
            return None
    ps = tower_params(model)
    ok = all(p.requires_grad and p.dtype == torch.float32 and p.is_contiguous() for p in ps)
    return ps if ok else None


_ADDLN_ON = os.environ.get("RSX_LINEAR_ADDLN", "1") != "0"


class _TowerPacked(torch.autograd.Function):
    """out = normalize(output_proj(...encoder(seq_embed(item_proj(pv)))...)) over packed tokens; see
    rsx_tower_fwd. Inputs with gradients: pv (optional), gate, profile and the tower parameters."""

    @staticmethod
    def forward(ctx, pv, gate, profile, cfg, *params):
        packed, tok_ids, p_drop, eps, nl, tail_last = cfg
        T, D = pv.shape
        U = packed.seg_off.numel() - 1
        dev = pv.device
        pv = _c(pv)
        gate = _c(gate)
        profile = _c(profile)
        perm, cb, chunk_ids, ch_off, uniq = packed.item_seg
        inputs = ([pv] + list(tok_ids) + [packed.tok_pos, packed.tok_pad, packed.seg_off, packed.seg_off64,
                                            packed.tok_user, gate, profile, perm, cb, chunk_ids, ch_off, uniq])
        tail_last = None if tail_last is None else _c(tail_last)
        ptrs = N.ptr_array(inputs + list(params) + [tail_last])
        tabs = params[2:8]
        tB = 0 if tail_last is None else tail_last.numel()
        R = T // 2 + tB if tB else T
        dims = N.i64_array([T, U, params[8].shape[0], nl, chunk_ids.numel(), uniq.numel()]
                           + [t.shape[0] for t in tabs] + [tB, T // 2])
        fargs = (ctypes.c_float * (len(eps) + 1))(p_drop, *eps)
        seeds = [next_seed() if p_drop > 0 else 0 for _ in range(1 + 4 * nl)]
        seeds_arr = (ctypes.c_uint64 * len(seeds))(*seeds)
        nbytes = N.lib().rsx_tower_arena_bytes(T, U, nl)
        arena = torch.empty(nbytes, device=dev, dtype=torch.uint8)
        out = torch.empty(R, D, device=dev, dtype=torch.float32)
        with timed("tower_fwd"):
            rc = N.lib().rsx_tower_fwd(ptrs, dims, fargs, seeds_arr, N.ptr(arena), nbytes, N.ptr(out), N.stream())
        N.check(rc, "tower_fwd")
        ctx.save_for_backward(pv, gate, profile, out, *params)
        ctx.keep = (inputs + [tail_last], arena, ptrs, dims, fargs, seeds_arr)
        ctx.shape = (T, U, params[8].shape[0], nl, chunk_ids.numel())
        return out

    @staticmethod
    def backward(ctx, dout):
        if ctx.keep is None:  # the arena (the forward's activations) is released by the first backward
            raise RuntimeError("tower_packed: a second backward through the same forward (retain_graph=True) "
                               "is not supported; run the forward again")
        pv, gate, profile, out, *params = ctx.saved_tensors
        inputs, arena, ptrs, dims, fargs, seeds_arr = ctx.keep
        T, U, L, nl, C = ctx.shape
        dev = dout.device
        dout = _c(dout)
        # accumulated: the six tables, pos_emb, emb_ln w / b, the gate (one zero-filled allocation);
        # written: every other parameter's gradient and the profile's
        acc_like = [gate] + [params[i] for i in range(2, 11)]
        dgate, *acc = _zeros_group(acc_like)
        written = _empty_group([params[0], params[1]] + list(params[11:]) + [profile])
        dprofile = written[-1]
        dparams = [written[0], written[1]] + acc + written[2:-1]
        dpv = torch.empty_like(pv) if ctx.needs_input_grad[0] else None
        grads = [dpv] + [None] * 11 + [dgate, dprofile] + [None] * 5 + dparams + [None]
        nws = N.lib().rsx_tower_bwd_workspace_bytes(T, U, L, nl, C)
        ws = torch.empty(nws, device=dev, dtype=torch.uint8)
        with timed("tower_bwd"):
            rc = N.lib().rsx_tower_bwd(ptrs, dims, fargs, seeds_arr, N.ptr(arena), N.ptr(out), N.ptr(dout),
                                       N.ptr_array(grads), N.ptr(ws), nws, N.stream())
        N.check(rc, "tower_bwd")
        ctx.keep = None
        return (dpv, dgate, dprofile, None) + tuple(dparams)


def _empty_group(likes):
    """Uninitialised fp32 buffers shaped like each tensor (None -> None), carved out of ONE
    allocation (16-B aligned slices)."""
    sizes = [0 if t is None else (t.numel() + 3) // 4 * 4 for t in likes]
    if sum(sizes) == 0:
        return [None] * len(likes)
    ref = next(t for t in likes if t is not None)
    flat = torch.empty(sum(sizes), device=ref.device, dtype=torch.float32)
    out, o = [], 0
    for t, n in zip(likes, sizes):
        out.append(None if t is None else flat[o:o + t.numel()].view(t.shape))
        o += n
    return out


def tower_packed(model, packed, pv_tok, tok_ids, s_g, profile, p_drop, params=None, tail_last=None):
    """The native form of SASRecUserTower.forward_packed after the static profile: [T, 128], or with
    tail_last (view 1's "last" token per user, [B]) the [T/2 + B, 128] tail rows (see
    rsx_tower_fwd). params: tower_native_ok's list (else rebuilt)."""
    layers = model.transformer_encoder.layers
    eps = [model.emb_ln.eps]
    for layer in layers:
        eps += [layer.norm1.eps, layer.norm2.eps]
    eps.append(model.output_proj[1].eps)
    cfg = (packed, [_c(t) for t in tok_ids], float(p_drop), [float(e) for e in eps], len(layers), tail_last)
    return _TowerPacked.apply(pv_tok, s_g, profile, cfg, *(params if params is not None else tower_params(model)))


# ----------------------------------------------------------------------------------------
# A9: item-tower RE fields over packed (valid) tokens
@torch.no_grad()
def bert_embed_packed(embeddings, ids, tok_pos):
    """BertEmbeddings(input_ids) rows for a packed token list (ids [T], positions tok_pos [T],
    token type 0) via rsx_embed3_ln; dropout as the module's (active only in training)."""
    N.ensure_device(ids)
    word = embeddings.word_embeddings.weight
    D = word.shape[1]
    T = ids.numel()
    out = torch.empty(T, D, device=ids.device, dtype=torch.float32)
    ln = embeddings.LayerNorm
    rc = N.lib().rsx_embed3_ln(N.ptr(word), word.stride(0), N.ptr(_c(embeddings.position_embeddings.weight)),
                               N.ptr(_c(embeddings.token_type_embeddings.weight[0])), N.ptr(ln.weight),
                               N.ptr(ln.bias), float(ln.eps), N.ptr(_c(ids)), N.ptr(_c(tok_pos)), T, D, N.ptr(out),
                               N.stream())
    N.check(rc, "embed3_ln")
    if embeddings.training and embeddings.dropout.p > 0:
        out = torch.nn.functional.dropout(out, embeddings.dropout.p, True)
    return out


class _SegmentMean(torch.autograd.Function):
    """vec[u] = sum_{t in [seg[u], seg[u+1])} x[t] / max(cnt[u], 1e-9): the masked mean of the
    reference's (feats * m).sum(1) / clamp(m.sum(1), 1e-9) over packed valid tokens."""

    @staticmethod
    def forward(ctx, x, seg, tok_seg, inv):
        U = inv.numel()
        D = x.shape[1]
        s = torch.empty(U, D, device=x.device, dtype=torch.float32)
        rc = N.lib().rsx_segment_sum_rows(N.ptr(x), x.stride(0), None, N.ptr(seg), None, U, D, None, -1, N.ptr(s),
                                          s.stride(0), 0, N.stream())
        N.check(rc, "segment_sum_rows(mean)")
        ctx.save_for_backward(tok_seg, inv)
        return s * inv.unsqueeze(1)

    @staticmethod
    def backward(ctx, dv):
        tok_seg, inv = ctx.saved_tensors
        return gather_rows(_c(dv * inv.unsqueeze(1)), tok_seg), None, None, None


def segment_mean(x, seg, tok_seg, counts):
    """x [T, D] packed rows (segments contiguous), seg [U+1] int64 offsets, tok_seg [T] int64,
    counts [U] float -> [U, D] means (a zero-count segment gives 0, as the clamp does)."""
    inv = 1.0 / torch.clamp(counts, min=1e-9)
    return _SegmentMean.apply(_c(x), _c(seg), _c(tok_seg), inv.float())


# ----------------------------------------------------------------------------------------
# DCN-V2 reranker: cross network + the cross half of the final head
def crossnet(x, kernels, biases, w_head=None, want_x=False):
    """rsx_crossnet: x [B, D] -> (x_L [B, D] or None, head_part [B] = x_L . w_head or None)."""
    N.ensure_device(x)
    x = _c(x)
    B, D = x.shape
    x_out = torch.empty(B, D, device=x.device, dtype=torch.float32) if want_x else None
    part = torch.empty(B, device=x.device, dtype=torch.float32) if w_head is not None else None
    rc = N.lib().rsx_crossnet(N.ptr(x), x.stride(0), B, D, len(kernels),
                              N.ptr_array([_c(k.reshape(-1)) for k in kernels]),
                              N.ptr_array([_c(b.reshape(-1)) for b in biases]),
                              N.ptr(None if w_head is None else _c(w_head.reshape(-1))), N.ptr(x_out), N.ptr(part),
                              N.stream())
    N.check(rc, "crossnet")
    return x_out, part


# ----------------------------------------------------------------------------------------
# A16: DeepFM forward (inference)
ACT_NONE, ACT_RELU, ACT_GELU = 0, 1, 2


def linear(x, weight, bias=None, act=ACT_NONE):
    """act(x @ weight.T + bias) on the fp32 MFMA (forward only). x [M, K], weight [N<=256, K]."""
    N.ensure_device(x)
    x = _c(x)
    M, K = x.shape
    n = weight.shape[0]
    y = torch.empty(M, n, device=x.device, dtype=torch.float32)
    with timed("linear"):
        rc = N.lib().rsx_linear_fwd(N.ptr(x), x.stride(0), N.ptr(_c(weight)), N.ptr(bias), M, n, K, act, N.ptr(y),
                                    N.stream())
    N.check(rc, "linear_fwd")
    return y


# RSX_DEEPFM_FUSED=0 selects the three-kernel path (gather+FM, fp32-MFMA linears) for A/B runs
_DEEPFM_FUSED = os.environ.get("RSX_DEEPFM_FUSED", "1") != "0"
# packed inference tables for the persistent DeepFM kernel (RSX_DEEPFM_PACK=0: read V / W directly)
_DEEPFM_PACK = os.environ.get("RSX_DEEPFM_PACK", "1") != "0"


class _FastKey:
    """Validity key of derived device state over a list of tensors: identities (the tensors are
    held, so an id cannot be recycled), storage pointers and in-place version counters, compared
    as three flat lists (≈ 0.25 µs per tensor; the per-tensor tuple key cost ≈ 0.75 µs)."""
    __slots__ = ("held", "ids", "ptrs", "vers")

    def __init__(self, ts):
        self.held = list(ts)
        self.ids = [id(t) for t in ts]
        self.ptrs = [t.data_ptr() for t in ts]
        self.vers = [t._version for t in ts]

    def matches(self, ts) -> bool:
        return ([id(t) for t in ts] == self.ids and [t._version for t in ts] == self.vers
                and [t.data_ptr() for t in ts] == self.ptrs)


def _deepfm_state(F, dev, emb_tables, lin_tables, dnn_weights, dnn_biases, w_out, cache):
    """Device state of the fused DeepFM kernel: the bf16 DNN weight images, the packed tables (when
    the kernel form takes them) and the pointer arrays, rebuilt when any input tensor changes
    (storage or in-place version). Kept in the caller's cache dict (the DeepFM module) between
    calls; without one it is built per call."""
    ts = list(emb_tables) + list(lin_tables) + list(dnn_weights) + list(dnn_biases) + [w_out]
    if cache is not None:
        st = cache.get("fused_state")
        if st is not None and st["dev"] == dev and st["key"].matches(ts):
            return st
    emb = [_c(t) for t in emb_tables]
    lin = [_c(t) for t in lin_tables]
    w1, w2 = _c(dnn_weights[0]), _c(dnn_weights[1])
    b1, b2 = _c(dnn_biases[0]), _c(dnn_biases[1])
    wo = _c(w_out.reshape(-1))
    ws = torch.empty(N.lib().rsx_deepfm_fused_workspace_bytes(F), device=dev, dtype=torch.uint8)
    N.check(N.lib().rsx_deepfm_fused_prep(F, N.ptr(w1), N.ptr(w2), N.ptr(ws), N.stream()), "deepfm_prep")
    packed = None
    if cache is not None and _DEEPFM_PACK and N.lib().rsx_deepfm_fused_uses_packed(F):
        # inference images of the tables: [vocab][32] per field (V row, W, pad); one 128-B line
        # per (row, field) instead of two
        packed = [torch.empty(v.shape[0], 32, device=dev, dtype=torch.float32) for v in emb]
        for v, w, p in zip(emb, lin, packed):
            N.check(N.lib().rsx_deepfm_pack(N.ptr(v), N.ptr(w), v.shape[0], N.ptr(p), N.stream()), "deepfm_pack")
    st = {"dev": dev, "key": _FastKey(ts), "hold": (emb, lin, w1, w2, b1, b2, wo, packed), "ws": N.ptr(ws),
          "ws_t": ws, "V": N.ptr_array(emb), "W": N.ptr_array(lin),
          "P": N.ptr_array(packed) if packed is not None else None,
          "b1": N.ptr(b1), "b2": N.ptr(b2), "wo": N.ptr(wo)}
    if cache is not None:
        cache["fused_state"] = st
    return st


def deepfm_forward(x, emb_tables, lin_tables, out_bias, dnn_weights, dnn_biases, w_out, cache=None):
    """DeepFM logits/probabilities for x [R, F] int64 (see csrc/deepfm.hip).

    emb_tables: F tensors [vocab_f, 16]; lin_tables: F tensors [vocab_f] (or [vocab_f, 1]);
    dnn_weights/dnn_biases: torch Linear layout, ReLU between layers; w_out [H_last].
    Config-3 shapes (E 16, DNN (256, 128)) run the single fused kernel (rsx_deepfm_fused, bf16x3
    DNN products); other shapes the gather + fp32-MFMA linear kernels. cache: a dict owned by the
    caller (the DeepFM module) that keeps the fused kernel's bf16 weight images between calls,
    rebuilt when either DNN weight changes (storage or in-place version). Returns (logit [R], prob [R])."""
    N.ensure_device(x)
    x = _c(x)
    R, F = x.shape
    E = emb_tables[0].shape[1]
    dev = x.device
    if (_DEEPFM_FUSED and E == 16 and F <= 64 and len(dnn_weights) == 2 and tuple(dnn_weights[0].shape) == (256, F * 16)
            and tuple(dnn_weights[1].shape) == (128, 256)):
        if len(emb_tables) != F or len(lin_tables) != F:
            raise ValueError(f"deepfm: {len(emb_tables)} embedding / {len(lin_tables)} linear tables for {F} fields")
        logit = torch.empty(R, device=dev, dtype=torch.float32)
        prob = torch.empty(R, device=dev, dtype=torch.float32)
        with timed("deepfm/fused"):
            st = _deepfm_state(F, dev, emb_tables, lin_tables, dnn_weights, dnn_biases, w_out, cache)
            rc = N.lib().rsx_deepfm_fused_run(N.ptr(x), R, F, st["V"], st["W"], st["P"], float(out_bias), st["b1"],
                                              st["b2"], st["wo"], st["ws"], N.ptr(logit), N.ptr(prob), N.stream())
        N.check(rc, "deepfm_fused")
        return logit, prob
    emb = torch.empty(R, F * E, device=dev, dtype=torch.float32)
    lin = torch.empty(R, device=dev, dtype=torch.float32)
    with timed("deepfm/embed"):
        rc = N.lib().rsx_deepfm_embed(N.ptr(x), R, F, E, N.ptr_array([_c(t) for t in emb_tables]),
                                      N.ptr_array([_c(t) for t in lin_tables]), float(out_bias), N.ptr(emb),
                                      N.ptr(lin), N.stream())
    N.check(rc, "deepfm_embed")
    h = emb
    for w, b in zip(dnn_weights[:-1], dnn_biases[:-1]):
        with timed("deepfm/linear"):
            y = torch.empty(R, w.shape[0], device=dev, dtype=torch.float32)
            rc = N.lib().rsx_linear_fwd(N.ptr(h), h.stride(0), N.ptr(_c(w)), N.ptr(b), R, w.shape[0], h.shape[1],
                                        ACT_RELU, N.ptr(y), N.stream())
        N.check(rc, "linear_fwd")
        h = y
    logit = torch.empty(R, device=dev, dtype=torch.float32)
    prob = torch.empty(R, device=dev, dtype=torch.float32)
    w, b = dnn_weights[-1], dnn_biases[-1]
    with timed("deepfm/linear_dot"):
        rc = N.lib().rsx_linear_dot_fwd(N.ptr(h), h.stride(0), N.ptr(_c(w)), N.ptr(b), R, w.shape[0], h.shape[1],
                                        ACT_RELU, N.ptr(_c(w_out.reshape(-1))), N.ptr(lin), N.ptr(logit),
                                        N.ptr(prob), N.stream())
    N.check(rc, "linear_dot_fwd")
    return logit, prob


# ----------------------------------------------------------------------------------------
# §8f #3: GDCN reranker batch (utils/data_preprocessing/feature_processor.py:144-195)
def reranker_batch(uidx, iidx, tables, max_len=50):
    """(dense [B,12] f32, cat [B], seq_ids [B,L], seq_mask [B,L], target [B]) of the batch rows
    uidx / iidx (int64 device row indices) from device tables (a dict: u_scaled [U,3] f32,
    u_raw [U,2] f64, u_cat [U], i_scaled [I,6] f32, i_raw [I,3] f64, i_num [I], seq_off [U+1],
    seq_ids [nnz]) on rsx_reranker_batch. L = the batch's longest min(len, max_len) (one host
    read of the per-row lengths: pad_sequence pads to the batch maximum)."""
    N.ensure_device(uidx)
    uidx, iidx = _c(uidx), _c(iidx)
    B = uidx.numel()
    dev = uidx.device
    t = tables
    lens = torch.empty(B, device=dev, dtype=torch.int64)
    N.check(N.lib().rsx_reranker_seq_lens(N.ptr(uidx), N.ptr(t["seq_off"]), B, int(max_len), N.ptr(lens), N.stream()),
            "reranker_seq_lens")
    L = int(lens.max().item()) if B > 0 else 0
    dense = torch.empty(B, 12, device=dev, dtype=torch.float32)
    cat = torch.empty(B, device=dev, dtype=torch.int64)
    target = torch.empty(B, device=dev, dtype=torch.int64)
    seq = torch.empty(B, L, device=dev, dtype=torch.int64)
    mask = torch.empty(B, L, device=dev, dtype=torch.int64)
    rc = N.lib().rsx_reranker_batch(
        N.ptr(uidx), N.ptr(iidx), B, N.ptr(t["u_scaled"]), N.ptr(t["u_raw"]), N.ptr(t["u_cat"]), N.ptr(t["i_scaled"]),
        N.ptr(t["i_raw"]), N.ptr(t["i_num"]), N.ptr(t["seq_off"]), N.ptr(t["seq_ids"]), int(max_len), L, N.ptr(dense),
        N.ptr(cat), N.ptr(target), N.ptr(seq), N.ptr(mask), N.stream())
    N.check(rc, "reranker_batch")
    return dense, cat, seq, mask, target


# ----------------------------------------------------------------------------------------
# A14: retrieval top-k
class IdRangeGuard:
    """Range check of embedding ids on the device without a host sync (rsx_ids_check): the call
    returns the ids with every out-of-range id replaced by 0 (the following gather stays in
    bounds) and copies a device flag into pinned host memory behind an event. The error is
    raised as IndexError by the next call whose flag is visible (a non-blocking event query) or
    by check(), which the callers run at their own synchronisation points -- like the
    asynchronous device-side assert an out-of-range nn.Embedding index raises on the
    reference's CUDA path."""

    def __init__(self, what):
        self.what = what
        self.pending = []

    def __call__(self, ids, n):
        self.poll()
        N.ensure_device(ids)
        ids = _c(ids.to(torch.int64))
        out = torch.empty_like(ids)
        flag = torch.zeros(1, device=ids.device, dtype=torch.int32)
        N.check(N.lib().rsx_ids_check(N.ptr(ids), ids.numel(), 0, int(n), N.ptr(out), N.ptr(flag), N.stream()),
                "ids_check")
        host = torch.empty(1, dtype=torch.int32, pin_memory=True)
        host.copy_(flag, non_blocking=True)
        ev = torch.cuda.Event()
        ev.record()
        self.pending.append((ev, host, flag, int(n)))
        return out

    def watch(self, flag, n=None):
        """Track a device int32 flag that a kernel sets for an out-of-range id (rsx_static_profile_fwd)
        in the same asynchronous way."""
        self.poll()
        host = torch.empty(1, dtype=torch.int32, pin_memory=True)
        host.copy_(flag, non_blocking=True)
        ev = torch.cuda.Event()
        ev.record()
        self.pending.append((ev, host, flag, n))

    def poll(self, wait=False):
        while self.pending and (wait or self.pending[0][0].query()):
            ev, host, _, n = self.pending.pop(0)
            ev.synchronize()
            if int(host[0]):
                self.pending.clear()
                rng = "its table's range" if n is None else f"[0, {n})"
                raise IndexError(f"{self.what}: id out of range {rng}")

    def check(self):
        """Raise for any call so far whose ids were out of range (waits for their checks)."""
        self.poll(wait=True)


# the static profile's nine lookups (v1_refine_usertower.py:472-481), checked inside prof_in_k
_STATIC_IDS = IdRangeGuard("static profile ids (SASRecUserTower's nine nn.Embedding lookups)")


_TOPK_PATHS = {0: "list", 1: "fast", 2: "bf16"}
_TOPK_CORPUS = {}


def _topk_corpus(it):
    """The bf16 corpus image of `it` for the single-scan path (rsx_topk_prepare_corpus), cached
    for the most recent corpus and rebuilt when it changes (identity, storage or in-place
    version, as DeepFM's images): retrieval corpora are static between calls (the serving
    index, evaluate_model's normalised item table), so the conversion pass runs once, not per
    call. A call on another stream waits for the image's build."""
    dev = it.device
    st = _TOPK_CORPUS.get(dev)
    if st is not None and st["key"].matches([it]):
        cur = torch.cuda.current_stream(dev)
        if cur != st["stream"]:
            cur.wait_event(st["event"])
            # the image is read on this stream too: its block must not return to the building
            # stream's pool (when the cache entry is replaced) before this stream's reads finish
            st["buf"].record_stream(cur)
        return st["buf"]
    NI = it.shape[0]
    buf = torch.empty(N.lib().rsx_topk_corpus_bytes(NI), device=dev, dtype=torch.uint8)
    with timed("retrieve_topk/prepare"):
        rc = N.lib().rsx_topk_prepare_corpus(N.ptr(it), it.stride(0), NI, N.ptr(buf), N.stream())
    N.check(rc, "topk_prepare_corpus")
    ev = torch.cuda.Event()
    ev.record()
    _TOPK_CORPUS[dev] = {"key": _FastKey([it]), "buf": buf, "event": ev,
                         "stream": torch.cuda.current_stream(dev)}
    return buf


def clear_retrieval_cache(device=None) -> None:
    """Drop the cached bf16 corpus image(s) (and the references to their corpora): about
    0.75 GB at 1M items. The next retrieval over a corpus rebuilds its image."""
    if device is None:
        _TOPK_CORPUS.clear()
    else:
        _TOPK_CORPUS.pop(torch.device(device), None)


def retrieve_topk(queries, items, k, diag=None):
    """(scores [Q, k] desc, indices [Q, k] int64) of queries @ items.T without materialising
    the score matrix. Ties resolve to the lower item index. D = 128.
    Large corpora take the bf16 single scan + exact fp32 rescoring (path "bf16"), whose corpus
    image is cached across calls (_topk_corpus). diag: optional dict; receives "path" ("list" /
    "fast" / "bf16"), "fallback" (bool) and "fallback_queries" (int): how many queries the
    path's exactness check sent to the exact list-based kernels (the "fast" path re-runs the
    whole batch; one host sync, for tests / diagnostics)."""
    N.ensure_device(queries)
    q = _c(queries.to(torch.float32))
    it = items if (items.stride(-1) == 1 and items.stride(0) % 4 == 0) else items.contiguous()
    Q, NI = q.shape[0], it.shape[0]
    path = N.lib().rsx_topk_path(Q, NI, k)
    corpus = _topk_corpus(it) if path == 2 and Q > 0 else None
    nws = (N.lib().rsx_topk_workspace_bytes_corpus(Q, NI, k) if corpus is not None
           else N.lib().rsx_topk_workspace_bytes(Q, NI, k))
    ws = torch.empty(nws, device=q.device, dtype=torch.uint8)
    sc = torch.empty(Q, k, device=q.device, dtype=torch.float32)
    ix = torch.empty(Q, k, device=q.device, dtype=torch.int64)
    with timed("retrieve_topk"):
        if corpus is not None:
            rc = N.lib().rsx_retrieve_topk_corpus(N.ptr(q), q.stride(0), N.ptr(it), it.stride(0), N.ptr(corpus), Q,
                                                  NI, k, N.ptr(ws), N.ptr(sc), N.ptr(ix), N.stream())
        else:
            rc = N.lib().rsx_retrieve_topk(N.ptr(q), q.stride(0), N.ptr(it), it.stride(0), Q, NI, k, N.ptr(ws),
                                           N.ptr(sc), N.ptr(ix), N.stream())
    N.check(rc, "retrieve_topk")
    if diag is not None:
        h = ws[:16].view(torch.int32).cpu().tolist()
        assert h[1] == path, (h, path)
        n = h[0] if path == 2 else (Q if (path == 1 and h[2]) else 0)
        diag["path"] = _TOPK_PATHS[path]
        diag["fallback"], diag["fallback_queries"] = n > 0, n
    return sc, ix


def hnm_mine(u_norm, i_norm, target_ids, k, hnm_threshold=0.90, temperature=1.0, ignored_at=None):
    """Hard-negative mining (v1_refine_usertower.py:641-669, 705-728, 776-790) in one kernel:
    per row the k largest of (u_norm @ i_norm.T) / temperature with same-target columns and
    columns whose item-item cosine exceeds hnm_threshold (off the diagonal) set to -inf.
    Returns (top_idx [N, k] int64, value desc then column asc; top_cos [N, k] raw cosines;
    avail [N] int32 = columns not ignored). No autograd (the reference mines under no_grad).
    ignored_at: optional [N, M] int64 column indices; then a 4th output [N, M] bool tells
    whether column ignored_at[i, m] is ignored for row i, read from the kernel's own masked
    workspace (the same item-item products and threshold test the mining used)."""
    N.ensure_device(u_norm)
    u = _c(u_norm.detach().to(torch.float32))
    it = _c(i_norm.detach().to(torch.float32))
    tg = _c(target_ids.to(torch.int64))
    n, d = u.shape
    if it.shape != u.shape or tg.shape != (n,):
        raise ValueError(f"hnm_mine: shapes {tuple(u.shape)} / {tuple(it.shape)} / {tuple(tg.shape)} disagree")
    if not 1 <= k <= n:
        raise ValueError(f"hnm_mine: k={k} out of range for N={n} (torch.topk would fail too)")
    if n > N.lib().rsx_hnm_max_rows():
        raise ValueError(f"hnm_mine: N={n} exceeds the LDS-resident row limit {N.lib().rsx_hnm_max_rows()}")
    idx = torch.empty(n, k, device=u.device, dtype=torch.int64)
    cos = torch.empty(n, k, device=u.device, dtype=torch.float32)
    avail = torch.empty(n, device=u.device, dtype=torch.int32)
    nws = N.lib().rsx_hnm_workspace_bytes(n)
    ws = torch.empty(nws, device=u.device, dtype=torch.uint8)
    with timed("hnm_mine"):
        rc = N.lib().rsx_hnm_mine(N.ptr(u), N.ptr(it), N.ptr(tg), n, d, k, float(hnm_threshold), float(temperature),
                                  N.ptr(ws), nws, N.ptr(idx), N.ptr(cos), N.ptr(avail), N.stream())
    N.check(rc, "hnm_mine")
    if ignored_at is None:
        return idx, cos, avail
    ldw = nws // (4 * n)
    masked = ws.view(torch.float32)[: n * ldw].view(n, ldw)
    return idx, cos, avail, torch.gather(masked, 1, ignored_at) == float("-inf")


# ----------------------------------------------------------------------------------------
# Optional per-op device timing (bench.py): HIP events on the launching (current) stream.
_TIMING = {"on": False, "events": {}}


class timed:
    def __init__(self, name):
        self.name = name

    def __enter__(self):
        if _TIMING["on"]:
            self.e0 = torch.cuda.Event(enable_timing=True)
            self.e0.record()
        return self

    def __exit__(self, *exc):
        if _TIMING["on"]:
            e1 = torch.cuda.Event(enable_timing=True)
            e1.record()
            _TIMING["events"].setdefault(self.name, []).append((self.e0, e1))
        return False


def timing_start():
    _TIMING["on"] = True
    _TIMING["events"] = {}


def timing_stop():
    """-> {name: (launches, total_ms)} (synchronises)."""
    _TIMING["on"] = False
    torch.cuda.synchronize()
    out = {}
    for k, evs in _TIMING["events"].items():
        out[k] = (len(evs), sum(a.elapsed_time(b) for a, b in evs))
    return out
