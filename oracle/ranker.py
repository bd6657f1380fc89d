"""CPU restatement of the reference's DCN-V2 re-ranker -- TEST INFRASTRUCTURE ONLY.

temp_model/ranker_skelet.py:239-357 (CrossNet, RankingModel, predict_for_user), dead code in
the reference (never instantiated there); restated in float64 from the source text.
Parity with the reference itself is UNPINNED (no fixtures; import denied).
"""
import torch
import torch.nn.functional as F


def crossnet(x, kernels, biases):
    """:258-272: x_l = x_0 * (x_l @ k + b) + x_l for each layer."""
    x0 = x
    xl = x
    for k, b in zip(kernels, biases):
        xl = x0 * (xl @ k.double() + b.double()) + xl
    return xl


def ranking_model_forward(model, user, item, context=None):
    """:313-338 in float64 with the model's parameters (eval: dropout off)."""
    x = torch.cat([user, item] + ([context] if context is not None else []), dim=1).double()
    cross = crossnet(x, [k for k in model.cross_net.kernels], [b for b in model.cross_net.biases])
    d = model.deep_net
    h = F.gelu(F.layer_norm(F.linear(x, d[0].weight.double(), d[0].bias.double()), (256,), d[1].weight.double(),
                            d[1].bias.double(), d[1].eps))
    h = F.gelu(F.layer_norm(F.linear(h, d[4].weight.double(), d[4].bias.double()), (128,), d[5].weight.double(),
                            d[5].bias.double(), d[5].eps))
    logits = F.linear(torch.cat([cross, h], 1), model.final_head.weight.double(), model.final_head.bias.double())
    return torch.sigmoid(logits)
