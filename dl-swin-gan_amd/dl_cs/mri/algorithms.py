"""Conjugate gradient for the HQS / MoDL solver (alg = dl_cs/mri/algorithms.py:11-73).

The normal operator A passed in runs on the HIP SENSE kernels; the CG vector
updates are device tensor ops (HQS is SURVEY 8(f) rank 3, not the PGD hot path).
"""
import torch
from torch import nn


class ConjugateGradient(nn.Module):
    """Solve A x = y for Hermitian positive-definite A with `num_iter` CG steps."""

    def __init__(self, A, num_iter, dbprint=False):
        super().__init__()
        self.A = A
        self.num_iter = num_iter
        self.dbprint = dbprint

    @staticmethod
    def zdot(x1, x2):
        return torch.sum(x1.conj() * x2)

    def zdot_single(self, x):
        return self.zdot(x, x).real

    def forward(self, x, y):
        r = y - self.A(x)
        rsold = self.zdot_single(r)
        p = r
        for i in range(self.num_iter):
            Ap = self.A(p)
            alpha = rsold / self.zdot(p, Ap)
            x = x + alpha * p
            r = r - alpha * Ap
            rsnew = self.zdot_single(r)
            p = (rsnew / rsold) * p + r
            rsold = rsnew
            if self.dbprint:
                print(f"CG Iteration {i}: {float(rsnew)}")
        return x
