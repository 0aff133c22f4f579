"""RD loss of the reference training script (examples/train.py:59-82).

bpp = sum_k sum(log lik_k) / (-ln2 * N*H*W); mse = mean((x_hat - x)^2);
loss = lmbda[q] * mse + bpp.  The forward is two HIP launches
(cai_rd_loss_fwd: every sum in one grid, then a fixed-order fold that forms
the three scalars), the backward one (cai_rd_loss_bwd).
"""
import torch.nn as nn

from . import _ops
from ._ops import RdLossFn, RdLossFnUnfused

LMBDA = [256, 512, 1024, 2048, 4096, 8192, 10240]   # train.py:65


class RateDistortionLoss(nn.Module):
    def __init__(self, q):
        super().__init__()
        self.lmbda = list(LMBDA)
        self.q = q

    def forward(self, output, target):
        N, _, H, W = target.size()
        liks = list(output["likelihoods"].values())
        fn = RdLossFnUnfused if _ops._RD_UNFUSED else RdLossFn
        loss, mse, bpp = fn.apply(output["x_hat"], target, float(self.lmbda[self.q]), N * H * W, *liks)
        return {"bpp_loss": bpp, "mse_loss": mse, "loss": loss}
