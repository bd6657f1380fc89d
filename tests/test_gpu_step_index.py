"""The device-built step index (rsx_step_index_*, csrc/step_index.hip) against the torch builders
it replaces (PackedTokens, pack_inputs, ops.sort_segments, ops.TargetGroups; dist.py with
RSX_DEVICE_INDEX=0): every array identical, element for element and in dtype, on edge-case and
full-size batches. The index is the per-batch host work of train_user_tower_all_time
(tower_code/v1_usertower_train.py:794-835) plus the grouped loss's target structures."""
import pytest
import torch

import recsys_amd  # noqa: F401
from recsys_amd import dist as D
from recsys_amd import synth
from tests.helpers import small_universe, to_dev

pytestmark = pytest.mark.gpu


def _build(batch, lookup, device_index):
    prev = D._DEVICE_INDEX
    D._DEVICE_INDEX = device_index
    try:
        ix = D.prepare_step_index(batch, pretrained_lookup=lookup)
    finally:
        D._DEVICE_INDEX = prev
    torch.cuda.synchronize()
    return ix


def _same(a, b, what):
    assert a.dtype == b.dtype, (what, a.dtype, b.dtype)
    assert a.shape == b.shape, (what, tuple(a.shape), tuple(b.shape))
    assert torch.equal(a, b), what


def _compare(batch, lookup):
    dv = _build(batch, lookup, True)
    tr = _build(batch, lookup, False)
    assert hasattr(dv, "wsb") and not hasattr(tr, "wsb")          # the device path really ran
    pk_d, pk2_d, ids_d, pv_d, st_d = dv.packed
    pk_t, pk2_t, ids_t, pv_t, st_t = tr.packed
    for f in ("flat", "tok_user", "tok_pos", "tok_pad", "seg_off", "seg_off64", "valid_tok", "last_tok"):
        _same(getattr(pk_d, f), getattr(pk_t, f), "pk." + f)
    for f in ("flat", "tok_user", "tok_pos", "tok_pad", "seg_off", "seg_off64"):
        _same(getattr(pk2_d, f), getattr(pk2_t, f), "pk2." + f)
    for k, (a, b) in enumerate(zip(pk2_d.item_seg, pk2_t.item_seg)):
        _same(a, b, f"item_seg[{k}]")
    for k, (a, b) in enumerate(zip(ids_d, ids_t)):
        _same(a, b, f"tok_ids[{k}]")
    _same(pv_d, pv_t, "pv_tok")
    for k, (a, b) in enumerate(zip(st_d, st_t)):
        _same(a, b, f"static[{k}]")
    assert dv.counts == tr.counts and dv.n_glob == tr.n_glob and dv.B == tr.B
    _same(dv.last_t, tr.last_t, "last_t")
    _same(dv.t_glob_last, tr.t_glob_last, "t_glob_last")
    if tr.groups is None:
        assert dv.groups is None
        return dv
    for f in ("uniq", "colcnt", "row_col", "row_beg", "row_end", "exc_cols", "exc_s", "exc_e", "exc_n", "col_beg",
              "col_end"):
        _same(getattr(dv.groups, f), getattr(tr.groups, f), "groups." + f)
    assert (dv.groups.n_rows, dv.groups.n_cols) == (tr.groups.n_rows, tr.groups.n_cols)
    return dv


@pytest.mark.parametrize("B,seed", [(64, 3), (257, 4)])
def test_step_index_matches_torch_small(gpu, B, seed):
    items = small_universe(500)
    batch = to_dev(synth.make_batch(items, B, seed=seed), gpu)
    _compare(batch, items.pretrained.to(gpu))


def test_step_index_edge_cases(gpu):
    """Users with no valid step (the whole row padding: one padded token at position 0), all 50
    valid, one valid, every target the same item, target 0 (the pad id) on a valid step (left
    padding throughout, as SASRecDataset produces it: PackedTokens' last_tok formula assumes it)."""
    items = small_universe(300)
    batch = synth.make_batch(items, 12, seed=9)
    pm = batch["padding_mask"]
    pm[0] = True                                  # no valid step
    pm[1] = False                                 # all valid
    pm[2] = True
    pm[2, -1] = False                             # one valid step
    pm[3] = False
    batch["target_ids"][3] = 17                   # one target repeated 50 times
    batch["target_ids"][4, -1] = 0                # target id 0 on a valid step
    pm[4, -1] = False
    for u in (6, 7, 8):                           # three users sharing targets
        pm[u, 30:] = False
        batch["target_ids"][u, 30:] = torch.arange(20) % 7 + 40
    dv = _compare(to_dev(batch, gpu), items.pretrained.to(gpu))
    assert dv.packed[0].seg_off[1] - dv.packed[0].seg_off[0] == 1   # user 0: the one padded token


def test_step_index_all_padding(gpu):
    """No valid step at all: no loss rows, no target columns (groups None), one token per user."""
    items = small_universe(100)
    batch = synth.make_batch(items, 16, seed=2)
    batch["padding_mask"][:] = True
    dv = _compare(to_dev(batch, gpu), items.pretrained.to(gpu))
    assert dv.n_glob == 0 and dv.groups is None and dv.packed[0].flat.numel() == 16


@pytest.mark.parametrize("B", [8192])
def test_step_index_full_size(gpu, B):
    """The headline batch (8192 users x 50, 47,062 items: ~153k rows, ~24k columns, ~158k tokens
    per view)."""
    items = synth.make_items(num_items=47_062, d=128, seed=0)
    batch = to_dev(synth.make_batch(items, B, seed=100), gpu)
    dv = _compare(batch, items.pretrained.to(gpu))
    assert dv.groups.n_cols > 20_000 and dv.n_glob > 150_000


def test_step_index_rejects_out_of_range_ids(gpu):
    items = small_universe(100)
    batch = to_dev(synth.make_batch(items, 8, seed=1), gpu)
    batch["target_ids"][2, -1] = 101              # the id domain is the lookup's 101 rows
    with pytest.raises(IndexError, match="outside"):
        D.prepare_step_index(batch, pretrained_lookup=items.pretrained.to(gpu))


@pytest.mark.parametrize("kind", ["width64", "fp16", "cpu", "requires_grad"])
def test_step_index_lookup_not_taken_by_device_builder(gpu, kind):
    """The device builder gathers 128-wide fp32 device rows itself (si_pv_k); any other pretrained
    lookup takes the torch builders: a 64-wide or fp16 one is gathered by ops.gather_rows as is, a
    lookup that requires grad keeps its autograd edge, a host lookup raises RuntimeError (no host
    pointer reaches a kernel)."""
    items = small_universe(100)
    batch = to_dev(synth.make_batch(items, 16, seed=3), gpu)
    lk = items.pretrained.to(gpu)
    if kind == "width64":
        lk = lk[:, :64].contiguous()
    elif kind == "fp16":
        lk = lk.half()
    elif kind == "cpu":
        lk = items.pretrained.clone()
    else:
        lk = lk.clone().requires_grad_()
    if kind == "cpu":
        with pytest.raises(RuntimeError):
            D.prepare_step_index(batch, pretrained_lookup=lk)
        return
    ix = D.prepare_step_index(batch, pretrained_lookup=lk)
    assert not hasattr(ix, "wsb")                      # the torch builders ran
    pk, _, ids, pv, _ = ix.packed
    exp = lk.float()[ids[0]] if kind != "requires_grad" else lk[ids[0]]
    torch.testing.assert_close(pv.float(), exp.float(), rtol=0, atol=0)
    if kind == "requires_grad":
        pv.sum().backward()
        assert lk.grad is not None and float(lk.grad.abs().sum()) > 0
