"""The rounding margin of the bf16 top-K filter (``ops.bf16_score_margin``), checked on the CPU.

``score_filter_bf16`` keeps item i for query q iff ``S_bf16 > theta - c |q| |x_i|``; exactness of
the scan rests on ``|S_bf16 - S_fp32| <= c |q| |x|``.  The bf16 products are exact in fp32, so
the worst case is the operand rounding; adversarial rows (every element just above a bf16
rounding boundary, all products of one sign) approach the bound, random rows stay far inside.
"""
import pytest
import torch

from flink_parameter_server_1_amd import ops


def _ratio(Q, X):
    exact = Q.double() @ X.double().T
    bf = Q.bfloat16().double() @ X.bfloat16().double().T  # products and sums exact in fp64
    fp32 = (Q @ X.T).double()
    bound = torch.linalg.vector_norm(Q.double(), dim=1)[:, None] * torch.linalg.vector_norm(X.double(), dim=1)[None]
    # the kernel compares against the fp32 MFMA score; both sides' fp32 accumulation is in c
    return float(((bf - fp32).abs() / bound).max()), float(((bf - exact).abs() / bound).max())


@pytest.mark.parametrize("D", [32, 64, 128])
def test_margin_bounds_random_rows(D):
    g = torch.Generator().manual_seed(D)
    Q = torch.randn(256, D, generator=g)
    X = torch.randn(2048, D, generator=g) * torch.rand(2048, 1, generator=g) * 3
    c = ops.bf16_score_margin(D)
    r32, rex = _ratio(Q, X)
    assert r32 <= c and rex <= c


@pytest.mark.parametrize("D", [32, 64, 128])
def test_margin_bounds_adversarial_rows(D):
    """Elements just below the midpoint between two bf16 values (1 + 2^-8 - 2^-20: rounded
    down by ~2^-8 relative, the worst case), equal signs so the errors add up: the ratio
    reaches ~2^-7, i.e. the bound is tight."""
    base = 1.0 + 2.0 ** -8 - 2.0 ** -20
    Q = torch.full((4, D), base)
    X = torch.full((4, D), base) * torch.tensor([1.0, 0.5, 2.0, 1.5]).view(-1, 1)
    c = ops.bf16_score_margin(D)
    r32, rex = _ratio(Q, X)
    assert rex > 0.95 * c  # the construction reaches the bound
    assert r32 <= c and rex <= c
