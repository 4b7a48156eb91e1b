"""centered_gram: second moments about the mean for narrow, far-from-zero features (latitude-like columns).

The raw-moment form E[x^2] - mean^2 of fp32 columns loses ~all digits of a variance of 4e-4 about 37.8; the
shifted Gram keeps them on both devices.  Reference: fp64 numpy.
"""
import numpy as np
import pytest
import torch

from cdnaml.models.util import centered_gram
from cdnaml.parallel.comm import Comm


def _devices():
    return ["cpu", pytest.param("cuda", marks=pytest.mark.gpu)]


@pytest.mark.parametrize("device", _devices())
def test_centered_gram_matches_fp64(device):
    rng = np.random.default_rng(3)
    n = 200_000
    X = np.stack([37.8 + 0.02 * rng.standard_normal(n), -122.4 + 0.03 * rng.standard_normal(n),
                  1e4 + 50 * rng.standard_normal(n), rng.standard_normal(n)], 1).astype(np.float32)
    Xd = X.astype(np.float64)
    n_, mean, C = centered_gram(torch.from_numpy(X).to(device), Comm(torch.device(device)))
    assert n_ == n
    np.testing.assert_allclose(mean.cpu().numpy(), Xd.mean(0), rtol=1e-9, atol=1e-6)
    Cref = (Xd - Xd.mean(0)).T @ (Xd - Xd.mean(0))
    np.testing.assert_allclose(np.diag(C.cpu().numpy()), np.diag(Cref), rtol=1e-4)
    np.testing.assert_allclose(C.cpu().numpy(), Cref, rtol=1e-4, atol=1e-4 * np.sqrt(np.outer(np.diag(Cref),
                                                                                               np.diag(Cref))).max())
