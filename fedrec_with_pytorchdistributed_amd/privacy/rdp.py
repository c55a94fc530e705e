"""Renyi-DP accountant for the Poisson-subsampled Gaussian mechanism + sigma calibration.

Replaces the reference's use of Opacus (``client.py:270-281``), which builds a private
model/optimizer/loader only to read ``noise_multiplier`` for a target (epsilon, delta)
over ``EPOCHS = 50`` epochs with sample rate ``batch_size / len(dataset)`` (Opacus uses
``1 / len(data_loader)``).  Opacus is not installed here, so this module re-derives the
same computation from the published analysis:

* RDP of the sampled Gaussian (Mironov, Talwar, Zhang 2019): integer orders by the
  binomial expansion, fractional orders by the two-sided erfc series;
* RDP -> (eps, delta) with the tightened conversion of Balle et al. 2020 (the one current
  Opacus uses): ``eps = rdp - (log delta + log a) / (a - 1) + log((a - 1) / a)``;
* default orders ``[1 + x/10 for x in 1..99] + [12..63]`` and the doubling + bisection
  search of ``get_noise_multiplier`` with epsilon tolerance 0.01.

Attribution: the structure of this module -- the log-space helpers ``_log_add`` / ``_log_sub``
/ ``_log_erfc``, the integer / fractional-order split ``_log_a_int`` / ``_log_a_frac``, the
``MAX_SIGMA`` cap and the doubling + bisection noise search with its "privacy budget is too
low" error -- follows the public Apache-2.0 RDP analysis of TensorFlow Privacy
(``rdp_accountant.py``) and Opacus (``opacus/accountants/analysis/rdp.py``,
``opacus/accountants/utils.py``), re-implemented here; the reference itself has no accountant.

Numerics are validated in tests against q = 1 (closed form ``a / (2 sigma^2)``) and
against direct numerical integration of the Renyi divergence; parity with the Opacus
package itself is unpinned (not importable offline).
"""
from __future__ import annotations

import math
from typing import List, Sequence, Tuple

import numpy as np
from scipy import special

DEFAULT_ALPHAS: List[float] = [1 + x / 10.0 for x in range(1, 100)] + list(range(12, 64))
MAX_SIGMA = 1e6


def _log_add(a: float, b: float) -> float:
    lo, hi = min(a, b), max(a, b)
    if lo == -np.inf:
        return hi
    return math.log1p(math.exp(lo - hi)) + hi


def _log_sub(a: float, b: float) -> float:
    if a < b:
        raise ValueError("log_sub: a < b")
    if b == -np.inf:
        return a
    if a == b:
        return -np.inf
    try:
        return math.log(math.expm1(a - b)) + b
    except OverflowError:
        return a


def _log_erfc(x: float) -> float:
    return math.log(2) + special.log_ndtr(-x * 2 ** 0.5)


def _log_a_int(q: float, sigma: float, alpha: int) -> float:
    log_a = -np.inf
    for i in range(alpha + 1):
        log_coef = math.log(special.binom(alpha, i)) + i * math.log(q) + (alpha - i) * math.log(1 - q)
        log_a = _log_add(log_a, log_coef + (i * i - i) / (2 * sigma ** 2))
    return float(log_a)


def _log_a_frac(q: float, sigma: float, alpha: float) -> float:
    log_a0, log_a1 = -np.inf, -np.inf
    i = 0
    z0 = sigma ** 2 * math.log(1 / q - 1) + 0.5
    while True:
        coef = special.binom(alpha, i)
        log_coef = math.log(abs(coef))
        j = alpha - i
        log_t0 = log_coef + i * math.log(q) + j * math.log(1 - q)
        log_t1 = log_coef + j * math.log(q) + i * math.log(1 - q)
        log_e0 = math.log(0.5) + _log_erfc((i - z0) / (math.sqrt(2) * sigma))
        log_e1 = math.log(0.5) + _log_erfc((z0 - j) / (math.sqrt(2) * sigma))
        log_s0 = log_t0 + (i * i - i) / (2 * sigma ** 2) + log_e0
        log_s1 = log_t1 + (j * j - j) / (2 * sigma ** 2) + log_e1
        if coef > 0:
            log_a0 = _log_add(log_a0, log_s0)
            log_a1 = _log_add(log_a1, log_s1)
        else:
            log_a0 = _log_sub(log_a0, log_s0)
            log_a1 = _log_sub(log_a1, log_s1)
        i += 1
        if max(log_s0, log_s1) < -30:
            break
    return _log_add(log_a0, log_a1)


def _rdp_one(q: float, sigma: float, alpha: float) -> float:
    if q == 0:
        return 0.0
    if sigma == 0:
        return np.inf
    if q == 1.0:
        return alpha / (2 * sigma ** 2)
    if np.isinf(alpha):
        return np.inf
    if float(alpha).is_integer():
        return _log_a_int(q, sigma, int(alpha)) / (alpha - 1)
    return _log_a_frac(q, sigma, alpha) / (alpha - 1)


def compute_rdp(q: float, noise_multiplier: float, steps: int, orders: Sequence[float]) -> np.ndarray:
    return np.array([_rdp_one(q, noise_multiplier, a) for a in orders]) * steps


def get_privacy_spent(orders: Sequence[float], rdp: np.ndarray, delta: float) -> Tuple[float, float]:
    orders_vec = np.atleast_1d(np.asarray(orders, dtype=np.float64))
    rdp_vec = np.atleast_1d(rdp)
    eps = rdp_vec - (np.log(delta) + np.log(orders_vec)) / (orders_vec - 1) + np.log((orders_vec - 1) / orders_vec)
    if np.isnan(eps).all():
        return np.inf, np.nan
    idx = int(np.nanargmin(eps))
    return float(eps[idx]), float(orders_vec[idx])


class RDPAccountant:
    def __init__(self):
        self.history: List[Tuple[float, float, int]] = []  # (sigma, q, steps)

    def step(self, noise_multiplier: float, sample_rate: float, steps: int = 1) -> None:
        if self.history and self.history[-1][:2] == (noise_multiplier, sample_rate):
            s, q, n = self.history[-1]
            self.history[-1] = (s, q, n + steps)
        else:
            self.history.append((noise_multiplier, sample_rate, steps))

    def get_epsilon(self, delta: float, alphas: Sequence[float] = DEFAULT_ALPHAS) -> float:
        rdp = sum(compute_rdp(q, s, n, alphas) for s, q, n in self.history) if self.history else np.zeros(len(alphas))
        return get_privacy_spent(alphas, rdp, delta)[0]


def get_noise_multiplier(target_epsilon: float, target_delta: float, sample_rate: float, epochs: float = None,
                         steps: int = None, epsilon_tolerance: float = 0.01) -> float:
    if steps is None:
        if epochs is None:
            raise ValueError("need epochs or steps")
        steps = int(epochs / sample_rate)
    eps_high = float("inf")
    sigma_low, sigma_high = 0.0, 10.0
    while eps_high > target_epsilon:
        sigma_high = 2 * sigma_high
        acc = RDPAccountant()
        acc.history = [(sigma_high, sample_rate, steps)]
        eps_high = acc.get_epsilon(target_delta)
        if sigma_high > MAX_SIGMA:
            raise ValueError("The privacy budget is too low.")
    while target_epsilon - eps_high > epsilon_tolerance:
        sigma = (sigma_low + sigma_high) / 2
        acc = RDPAccountant()
        acc.history = [(sigma, sample_rate, steps)]
        eps = acc.get_epsilon(target_delta)
        if eps < target_epsilon:
            sigma_high = sigma
            eps_high = eps
        else:
            sigma_low = sigma
    return sigma_high


def calibrate_client_sigma(epsilon: float, delta: float, batch_size: int, n_train: int, epochs: int) -> float:
    """Mirror of ``make_private_with_epsilon`` at ``client.py:271-279`` (sample rate =
    1 / number of batches of the client's loader)."""
    n_batches = max(1, -(-n_train // batch_size))
    return get_noise_multiplier(epsilon, delta, 1.0 / n_batches, epochs=epochs)
