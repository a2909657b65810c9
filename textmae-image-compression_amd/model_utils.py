"""Optimizer split — counterpart of reference models/Compression/common/model_utils.py:67-90:
Adam over every trainable parameter except ``*.quantiles``; a second (aux) Adam over ``*.quantiles``."""
import torch.optim as optim


def configure_optimizers(model, args):
    parameters = {n for n, p in model.named_parameters() if not n.endswith(".quantiles") and p.requires_grad}
    aux_parameters = {n for n, p in model.named_parameters() if n.endswith(".quantiles") and p.requires_grad}
    params = dict(model.named_parameters())
    assert not (parameters & aux_parameters)
    optimizer = optim.Adam((params[n] for n in sorted(parameters)), lr=args.learning_rate)
    aux_optimizer = optim.Adam((params[n] for n in sorted(aux_parameters)), lr=args.aux_learning_rate)
    return optimizer, aux_optimizer
