"""CPU restatement of DeepFM (BASELINE configs[2]) -- TEST INFRASTRUCTURE ONLY.

The reference has no DeepFM (SURVEY.md §0 finding 1): it pins deepctr-torch==0.2.9
(requirements.txt:41) but never imports it, and the library is absent here. This follows the
library's published formulation: linear part (per-field 1-d embeddings, summed) + FM
(0.5 * sum_k[(sum_f v)^2 - sum_f v^2], deepctr FM.forward) + DNN (Linear+ReLU stack, then
dnn_linear without bias) + PredictionLayer bias, sigmoid. PARITY UNPINNED (no reference
code, fixtures or library to compare against).
"""
import torch
import torch.nn.functional as F


def deepfm_forward(x, emb_tables, lin_tables, out_bias, dnn_weights, dnn_biases, w_out, dtype=torch.float64):
    """x [R, F] int64 -> (logit [R], prob [R]) in `dtype` (float64 for the parity tests; float32,
    the reference arithmetic, for bench.py's CPU baseline) on the CPU. Rows are gathered before
    the conversion (the same values as converting the tables)."""
    emb = torch.stack([t[x[:, f]].to(dtype) for f, t in enumerate(emb_tables)], dim=1)      # [R, F, E]
    linear = sum(t.reshape(-1)[x[:, f]].to(dtype) for f, t in enumerate(lin_tables))        # [R]
    square_of_sum = emb.sum(dim=1) ** 2
    sum_of_square = (emb * emb).sum(dim=1)
    fm = 0.5 * (square_of_sum - sum_of_square).sum(dim=1)
    h = emb.reshape(emb.shape[0], -1)
    for w, b in zip(dnn_weights, dnn_biases):
        h = F.relu(h @ w.to(dtype).T + b.to(dtype))
    dnn = h @ w_out.to(dtype).reshape(-1)
    logit = out_bias + linear + fm + dnn
    return logit, torch.sigmoid(logit)
