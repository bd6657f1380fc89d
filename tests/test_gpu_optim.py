"""rsx_clip_adamw (ops.clip_adamw_step): clip_grad_norm_ + torch.optim.AdamW.step in two launches,
checked against torch's own pair on the same tensors (tower_code/v1_usertower_train.py:852-853:
clip the user tower's gradients to norm 5, AdamW over the tower and, at lr x 0.05, the item matrix).

Tolerances: against torch's fused AdamW (whose double-precision scalar arithmetic the kernel
follows) parameters within rtol 5e-7 (a few ulp; 8 of 6M elements differ by one ulp), against the
foreach AdamW (float lerp / addcdiv forms, CPU step counts) rtol 1e-6 / atol 1e-7 (2e-4 of one
step's update); clipped gradients and the total norm within 1e-6 relative (the norm is summed in
a different order)."""
import copy

import pytest
import torch

from recsys_amd import ops

pytestmark = pytest.mark.gpu

# sizes: > one 8192-element tile, not a multiple of 4 (scalar path), a 0-d scalar, an empty tensor
_SIZES = [(47063, 128), (128,), (3, 7), (), (0, 5), (384, 128), (33,), (100, 128)] + [(16,)] * 30


def _setup(seed, fused, grad_scale, n_item=1):
    g = torch.Generator(device="cuda").manual_seed(seed)
    tower = [torch.nn.Parameter(torch.randn(s, device="cuda", generator=g) * 0.1) for s in _SIZES]
    items = [torch.nn.Parameter(torch.randn(1000, 128, device="cuda", generator=g)) for _ in range(n_item)]

    def grads():
        for p in tower + items:
            p.grad = torch.randn(p.shape, device="cuda", generator=g) * grad_scale

    opt = torch.optim.AdamW(tower, lr=5e-4, weight_decay=0.01, fused=fused)
    opt.add_param_group({"params": items, "lr": 5e-4 * 0.05})
    return tower, items, grads, opt


def _clone(tower, items, opt, fused):
    t2 = [torch.nn.Parameter(p.detach().clone()) for p in tower]
    i2 = [torch.nn.Parameter(p.detach().clone()) for p in items]
    o2 = torch.optim.AdamW(t2, lr=5e-4, weight_decay=0.01, fused=fused)
    o2.add_param_group({"params": i2, "lr": 5e-4 * 0.05})
    o2.load_state_dict(copy.deepcopy(opt.state_dict()))
    return t2, i2, o2


@pytest.mark.parametrize("fused,grad_scale", [(True, 1.0), (True, 1e-4), (None, 1.0)])
def test_clip_adamw_matches_torch(fused, grad_scale):
    tower, items, grads, opt = _setup(0, fused, grad_scale)
    t2, i2, o2 = _clone(tower, items, opt, fused)
    rtol, atol = (5e-7, 1e-9) if fused else (1e-6, 1e-7)
    for step in range(3):
        grads()
        for a, b in zip(tower + items, t2 + i2):
            b.grad = a.grad.clone()
        norm = ops.clip_adamw_step(opt, tower, 5.0)
        assert norm is not None
        ref_norm = torch.nn.utils.clip_grad_norm_(t2, max_norm=5.0)
        o2.step()
        torch.testing.assert_close(norm, ref_norm, rtol=1e-6, atol=0)
        if grad_scale >= 1.0:
            assert float(ref_norm) > 5.0   # the clip is active
        for a, b in zip(tower + items, t2 + i2):
            torch.testing.assert_close(a.grad, b.grad, rtol=1e-6, atol=1e-12)
            torch.testing.assert_close(a.detach(), b.detach(), rtol=rtol, atol=atol)
        for a, b in zip(tower + items, t2 + i2):
            sa, sb = opt.state[a], o2.state[b]
            assert float(sa["step"]) == float(sb["step"]) == step + 1
            assert sa["step"].device == sb["step"].device
            # foreach AdamW forms exp_avg by lerp in float: ~3e-8 absolute on O(0.1) moments
            torch.testing.assert_close(sa["exp_avg"], sb["exp_avg"], rtol=1e-5, atol=1e-9 if fused else 1e-7)
            torch.testing.assert_close(sa["exp_avg_sq"], sb["exp_avg_sq"], rtol=1e-5, atol=1e-12)


def test_clip_adamw_state_interchangeable_with_torch():
    """Two native steps, then torch's own step continues from the same state (and vice versa):
    the state entries are the ones torch.optim.AdamW creates and reads."""
    tower, items, grads, opt = _setup(1, True, 1.0)
    t2, i2, o2 = _clone(tower, items, opt, True)
    for step in range(4):
        grads()
        for a, b in zip(tower + items, t2 + i2):
            b.grad = a.grad.clone()
        if step in (0, 1):
            assert ops.clip_adamw_step(opt, tower, 5.0) is not None
        else:
            torch.nn.utils.clip_grad_norm_(tower, max_norm=5.0)
            opt.step()
        torch.nn.utils.clip_grad_norm_(t2, max_norm=5.0)
        o2.step()
    for a, b in zip(tower + items, t2 + i2):
        torch.testing.assert_close(a.detach(), b.detach(), rtol=1e-6, atol=1e-7)


def test_clip_adamw_skips_params_without_grad_and_declines_others():
    tower, items, grads, opt = _setup(2, True, 1.0)
    grads()
    tower[1].grad = None
    assert ops.clip_adamw_step(opt, tower, 5.0) is not None
    assert len(opt.state[tower[1]]) == 0 and float(opt.state[tower[0]]["step"]) == 1.0
    # a clipped parameter the optimizer does not own, SGD, amsgrad: declined, nothing changed
    stray = torch.nn.Parameter(torch.zeros(4, device="cuda"))
    stray.grad = torch.ones(4, device="cuda")
    p0 = tower[0].detach().clone()
    assert ops.clip_adamw_step(opt, tower + [stray], 5.0) is None
    assert torch.equal(tower[0].detach(), p0)
    assert ops.clip_adamw_step(torch.optim.SGD(tower, lr=0.1), tower, 5.0) is None
    assert ops.clip_adamw_step(torch.optim.AdamW(tower, amsgrad=True), tower, 5.0) is None
