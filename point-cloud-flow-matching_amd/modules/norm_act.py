"""BatchNorm (training-mode batch statistics) fused with the activation that
follows it on the PVConv path: SharedMLP's BN1d + ReLU
(third_party/pvcnn/modules/shared_mlp.py:15-27) and PVConv's BN3d +
LeakyReLU(0.1) (third_party/pvcnn/modules/pvconv.py:20-30).

`bn_act(x, bn, slope)` computes act(bn(x)) with the nn.BatchNorm module's own
parameters and buffers: on a HIP device in training mode it runs pcfm's fused
kernels (csrc/norm.hip; running_mean / running_var / num_batches_tracked
updated as torch does); otherwise (eval mode, CPU, momentum=None) the module
and the activation run as in the reference.
"""
import torch
import torch.nn.functional as F

__all__ = ["bn_act", "gn_film_residual"]


class _BNAct(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, weight, bias, running_mean, running_var, eps, momentum, slope):
        from pcfm import ops
        y, mean, invstd = ops.bn_act_forward(x, weight, bias, eps, slope, momentum, running_mean,
                                             running_var)
        ctx.save_for_backward(x, weight, bias, mean, invstd)
        ctx.slope = slope
        return y

    @staticmethod
    def backward(ctx, dy):
        from pcfm import ops
        x, weight, bias, mean, invstd = ctx.saved_tensors
        dx, dgamma, dbeta = ops.bn_act_backward(dy, x, weight, bias, mean, invstd, ctx.slope)
        return dx, dgamma, dbeta, None, None, None, None, None


def _fusable(x: torch.Tensor, bn) -> bool:
    if not (x.is_cuda and x.dtype == torch.float32 and x.dim() >= 3 and bn.training
            and bn.affine and bn.track_running_stats and bn.momentum is not None
            and bn.running_mean is not None and not torch.is_autocast_enabled("cuda")):
        return False
    s = x[0, 0].numel()
    return s % 4 == 0 and x.shape[0] * x.shape[1] < 65536 and x.numel() > 0


def bn_act(x: torch.Tensor, bn, slope: float) -> torch.Tensor:
    """act(bn(x)) with act(v) = v if v > 0 else slope * v (slope 0: ReLU)."""
    if _fusable(x, bn):
        bn.num_batches_tracked.add_(1)
        return _BNAct.apply(x.contiguous(), bn.weight, bn.bias, bn.running_mean, bn.running_var,
                            float(bn.eps), float(bn.momentum), float(slope))
    y = bn(x)
    return F.relu(y, inplace=True) if slope == 0 else F.leaky_relu(y, slope, inplace=True)


class _GNFiLMRes(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, weight, bias, gamma, beta, groups, eps):
        from pcfm import ops
        out, mean, rstd = ops.gn_film_res_forward(x, weight, bias, gamma, beta, groups, eps)
        ctx.save_for_backward(x, weight, bias, gamma, mean, rstd)
        ctx.groups = groups
        return out

    @staticmethod
    def backward(ctx, dout):
        from pcfm import ops
        x, weight, bias, gamma, mean, rstd = ctx.saved_tensors
        dx, dw, db, dg, dbt = ops.gn_film_res_backward(dout, x, weight, bias, gamma, mean, rstd,
                                                       ctx.groups)
        return dx, dw, db, dg, dbt, None, None


def gn_film_residual(x: torch.Tensor, norm, gamma: torch.Tensor, beta: torch.Tensor):
    """x + (norm(x) * (1 + gamma[:, :, None]) + beta[:, :, None]) for a GroupNorm
    `norm` (reference models.py:322-368); fused on a HIP device in fp32."""
    fused = (x.is_cuda and x.dtype == torch.float32 and x.dim() == 3
             and isinstance(norm, torch.nn.GroupNorm) and norm.affine
             and x.shape[2] % 4 == 0 and x.shape[1] <= 1024 and x.shape[0] * x.shape[1] < 65536
             and gamma.dtype == torch.float32 and beta.dtype == torch.float32
             and not torch.is_autocast_enabled("cuda"))
    if fused:
        return _GNFiLMRes.apply(x.contiguous(), norm.weight, norm.bias, gamma, beta,
                                int(norm.num_groups), float(norm.eps))
    y = norm(x)
    return x + (y * (1.0 + gamma[:, :, None]) + beta[:, :, None])
