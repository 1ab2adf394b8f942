"""Linear binding (interim: hipBLASLt via F.linear until gemm.hip lands)."""
from .linear import linear_reference


def linear(x, w, b, act):
    return linear_reference(x, w, b, act)
