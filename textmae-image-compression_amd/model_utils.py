"""Optimizer split — counterpart of reference models/Compression/common/model_utils.py:67-90 with the
reference's signature ``configure_optimizers(model, args)``: Adam over every trainable parameter except
``*.quantiles``; a second (aux) Adam over ``*.quantiles``.  ``fused=True`` gives the HIP FusedAdam
(optim.py) — same torch.optim.Adam arithmetic and checkpoint format."""
from . import optim


def configure_optimizers(model, args, fused=False):
    return optim.configure_optimizers(model, lr=args.learning_rate, aux_lr=args.aux_learning_rate, fused=fused)
