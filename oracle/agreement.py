"""Agreement of one full contrastive train step (two views, LogQ + DuoRec losses, backward,
clip_grad_norm_(5.0), AdamW) between the oracle (oracle/user_tower.py contrastive_step, the restatement of
tower_code/v1_usertower_train.py:717-893 / :850-854) and the HIP path, from the same state on the same batch.

TEST INFRASTRUCTURE ONLY (oracle/__init__.py): used by tests/test_gpu_fullstep.py and by bench.py's
cpu_baseline leg, which runs this oracle step anyway and checks the GPU step against it instead of discarding
its result. Nothing here runs product code: the caller hands in CPU copies of both sides.

Criteria, per side a dict {"losses": (total, main, cl), "grads": {name: t}, "params":
{name: t}} with every user-tower parameter by its state_dict name plus "item_matrix" (the unfrozen item
table, lr x 0.05, not clipped: the reference clips model.parameters() only, :852):
  * total / main / cl within 1e-4 (absolute; north_star's logit tolerance);
  * every parameter gradient within 1e-3 of that gradient's scale (max |g_ref|), after clipping on both
    sides (the clip coefficient is one scalar per step);
  * post-AdamW parameters within 1e-5 absolute. AdamW divides each element's moment by the square root of
    its second moment, so an element whose gradient is itself unresolved at the gradient tolerance (|g_ref|
    below the allowed gradient error, e.g. exact cancellations) can move by up to ~lr either way; such
    elements are counted separately ("unresolved") and must be the only ones over 1e-5.
"""
from __future__ import annotations

import torch

LOSS_TOL = 1e-4
GRAD_TOL = 1e-3     # of each gradient's scale
PARAM_TOL = 1e-5


def capture(model, item_matrix, losses, item_name="item_matrix"):
    """CPU copies of one side's step result: losses, clipped gradients, post-step parameters."""
    grads, params = {}, {}
    for n, p in list(model.named_parameters()) + [(item_name, item_matrix)]:
        params[n] = p.detach().float().cpu().clone()
        grads[n] = (p.grad.detach().float().cpu().clone() if p.grad is not None else torch.zeros_like(params[n]))
    return {"losses": tuple(float(x) for x in losses), "grads": grads, "params": params}


def compare_step(ref, dut):
    """-> dict of the worst deviations and "ok" (every criterion of the module docstring)."""
    out = {"loss_abs_err": [abs(a - b) for a, b in zip(ref["losses"], dut["losses"])]}
    g_worst, g_name = 0.0, None
    p_worst, p_worst_resolved, n_over, n_unres_over, n_elems = 0.0, 0.0, 0, 0, 0
    for n, gr in ref["grads"].items():
        gd = dut["grads"][n]
        scale = float(gr.abs().max()) + 1e-30
        gerr = (gd - gr).abs()
        rel = float(gerr.max()) / scale
        if rel > g_worst:
            g_worst, g_name = rel, n
        pd = (dut["params"][n] - ref["params"][n]).abs()
        n_elems += pd.numel()
        # unresolved: the reference gradient is within the allowed gradient error of zero
        unres = gr.abs() <= GRAD_TOL * scale
        over = pd > PARAM_TOL
        n_over += int(over.sum())
        n_unres_over += int((over & unres).sum())
        p_worst = max(p_worst, float(pd.max()))
        if (~unres).any():
            p_worst_resolved = max(p_worst_resolved, float(pd[~unres].max()))
    out.update({"grad_max_err_over_scale": g_worst, "grad_worst_param": g_name,
                "param_max_abs_err": p_worst, "param_max_abs_err_resolved": p_worst_resolved,
                "params_over_1e-5": n_over, "params_over_1e-5_unresolved": n_unres_over, "param_elements": n_elems})
    out["ok"] = (max(out["loss_abs_err"]) <= LOSS_TOL and g_worst <= GRAD_TOL and p_worst_resolved <= PARAM_TOL
                 and n_over == n_unres_over)
    return out
