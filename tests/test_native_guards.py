"""Host-side argument guards of the HIP kernel bindings: out-of-range shapes must
raise before anything is launched (checked on CPU: the binding throws before any
HIP call, so null pointers are never dereferenced)."""
import pytest

from xgserve.ops._native import kernels


@pytest.mark.parametrize("E,k", [(65, 2), (0, 1), (8, 0), (8, 17), (4, 5), (128, 8)])
def test_moe_topk_softmax_rejects_out_of_range(E, k):
    with pytest.raises(ValueError):
        kernels().moe_topk_softmax(0, 1, 4, E, k, 1, 0, 0, 0)


def test_moe_align_rejects_out_of_range():
    with pytest.raises(ValueError):
        kernels().moe_align(0, 4, 2, 300, 0, 64, 0, 0, 0, 0)
