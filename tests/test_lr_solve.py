"""LinearRegression closed-form fast path (_solve_ridge: one Cholesky of the unscaled covariance) against the
general standardised solve, on a Gram of correlated features (OLS and ridge, with and without standardisation)."""
import numpy as np
import pytest

from cdnaml.models.regression import LinearRegression


@pytest.mark.parametrize("reg,std", [(0.0, True), (0.3, True), (0.3, False), (1e-3, True)])
def test_ridge_fast_path_matches_general_solve(monkeypatch, reg, std):
    rng = np.random.default_rng(1)
    d, m = 30, 5000
    Z = rng.standard_normal((m, d)) @ rng.standard_normal((d, d)) * rng.uniform(0.1, 10, d) + rng.uniform(-5, 5, d)
    y = Z @ rng.standard_normal(d) + 3 + rng.standard_normal(m)
    A = np.concatenate([Z, np.ones((m, 1)), y[:, None]], 1)
    G = A.T @ A
    lr = LinearRegression(regParam=reg, elasticNetParam=0.0, standardization=std)
    fast = lr._solve(G, d, np.zeros(d), 0.0)
    monkeypatch.setattr(LinearRegression, "_solve_ridge", lambda self, *a: None)
    ref = lr._solve(G, d, np.zeros(d), 0.0)
    np.testing.assert_allclose(fast[0], ref[0], rtol=1e-9, atol=1e-12)
    assert abs(fast[1] - ref[1]) <= 1e-9 * max(1.0, abs(ref[1]))
    np.testing.assert_allclose(fast[2], ref[2], rtol=1e-9)
    if reg == 0.0:
        np.testing.assert_allclose(fast[4](), ref[4](), rtol=1e-9)
